// Fused MobileNetV2 inverted-residual block for gfx950:
//   out = project( relu6( dw3x3( relu6( expand(x) ) ) ) ) [+ x]
// in ONE kernel, for the high-resolution blocks (257^2 / 129^2 / 65^2 maps) where
// the unfused pipeline is purely HBM-bound: the 6x-expanded tensor and the
// depthwise output never leave the CU.
//
// Workgroup = one (4*GPW) x 16 output tile of one image, 4 waves; wave w owns
// output rows GPW*w .. GPW*w+GPW-1 (16-pixel MFMA column groups).
//   1. The input tile with its halo ((8-1)*s+3) x ((16-1)*s+3) pixels x Cin is
//      staged once in LDS (zero outside the image and beyond Cin).
//   2. The hidden dimension is streamed in 32-channel chunks:
//      a. expand on MFMA (v_mfma_f32_16x16x32_bf16, A = expand weights,
//         B = input-tile pixels from LDS) + bias + ReLU6 -> LDS chunk E
//         (zeroed outside the image: the depthwise zero-padding applies to the
//         expanded tensor, not to relu6(bias));
//      b. 3x3 depthwise on the VALU from E: each lane computes 8 channels of one
//         output pixel, which is exactly its B fragment for the projection MFMA
//         (lane l: pixel l&15, channels 8*(l>>4)..+7), so the depthwise result
//         goes straight from registers into the MFMA;
//      c. project on MFMA into fp32 register accumulators.
//   3. Epilogue: + bias (+ residual read from the LDS input tile), bf16 store.
// Host-side packing pads Cin to a multiple of 32 and hid to a multiple of 32
// with zero weights, so every MFMA is full and no K masking is needed.
#include "common.h"
#include "kernels.h"

namespace ssa {
namespace {

constexpr int TW = 16;

struct IRArgs {
  const bf16* in;   // [B, IH, IW, Cin]
  const bf16* we;   // [hidP, CinP] (null: no expansion, hid == Cin)
  const float* be;  // [hidP]
  const float* wd;  // [9, hidP]
  const float* bd;  // [hidP]
  const bf16* wp;   // [CoutP, hidP]
  const float* bp;  // [CoutP]
  bf16* out;        // [B, OH, OW, Cout]
  int B, IH, IW, Cin, CinP, hidP, Cout, OH, OW, stride, residual;
};

template <int NSUB, bool EXPAND, int GPW>
__global__ __launch_bounds__(256) void fused_ir_kernel(IRArgs a) {
  constexpr int TH = 4 * GPW;  // wave w owns output rows GPW*w .. GPW*w + GPW-1
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = a.stride;
  const int TIH = (TH - 1) * s + 3, TIW = (TW - 1) * s + 3;
  const int in_px = TIH * TIW;
  const int in_groups = (in_px + 15) / 16;
  const int CinP = a.CinP;
  // LDS rows padded by 16 B: a 64-B (or 128-B) row stride puts the 16 lanes of a
  // ds_read_b128 group on 4 bank slots; +16 B spreads them over all 16.
  const int XS = CinP + 8, ES = 32 + 8;                   // row strides (elements)
  bf16* X = reinterpret_cast<bf16*>(smem);                // [in_groups*16][XS]
  bf16* E = X + (size_t)in_groups * 16 * XS;              // [in_groups*16][ES]

  const int tiles_x = cdiv_dev(a.OW, TW), tiles_y = cdiv_dev(a.OH, TH);
  const int b = blockIdx.x / (tiles_x * tiles_y);
  const int t = blockIdx.x % (tiles_x * tiles_y);
  const int oy0 = (t / tiles_x) * TH, ox0 = (t % tiles_x) * TW;
  const int iy0 = oy0 * s - 1, ix0 = ox0 * s - 1;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;

  // ---- 1. stage the input tile (16-byte chunks, zero outside image / Cin)
  const int cpp = CinP / 8;
  for (int i = tid; i < in_groups * 16 * cpp; i += 256) {
    const int ip = i / cpp, c = (i % cpp) * 8;
    const int ty = ip / TIW, tx = ip % TIW;
    const int iy = iy0 + ty, ix = ix0 + tx;
    bf16x8 v = zero8();
    if (ip < in_px && c < a.Cin && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW)
      v = ld8(a.in + (((long long)b * a.IH + iy) * a.IW + ix) * a.Cin + c);
    st8(X + (size_t)ip * XS + c, v);
  }
  __syncthreads();

  f32x4 acc[GPW][NSUB];
#pragma unroll
  for (int g = 0; g < GPW; ++g)
#pragma unroll
    for (int n = 0; n < NSUB; ++n) acc[g][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int hid = EXPAND ? a.hidP : CinP;
  for (int c0 = 0; c0 < hid; c0 += 32) {
    // ---- 2a. expand chunk -> E (MFMA), or alias the input channels
    if (EXPAND) {
      // chunk weights and biases: loop-invariant over the pixel groups
      bf16x8 wfr[2][2];
      float bias[2][4];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const bf16* wrow = a.we + (size_t)(c0 + sub * 16 + r16) * CinP;
        wfr[sub][0] = ld8(wrow + kq * 8);
        wfr[sub][1] = CinP > 32 ? ld8(wrow + 32 + kq * 8) : zero8();
        const float4 bv = *reinterpret_cast<const float4*>(a.be + c0 + sub * 16 + kq * 4);
        bias[sub][0] = bv.x; bias[sub][1] = bv.y; bias[sub][2] = bv.z; bias[sub][3] = bv.w;
      }
      for (int gi = wid; gi < in_groups; gi += 4) {
        const int ip = gi * 16 + r16;
        const int ty = ip / TIW, tx = ip - ty * TIW;
        const int iy = iy0 + ty, ix = ix0 + tx;
        const bool inside = ip < in_px && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
        const bf16x8 x0 = ld8(X + (size_t)ip * XS + kq * 8);
        const bf16x8 x1 = CinP > 32 ? ld8(X + (size_t)ip * XS + 32 + kq * 8) : zero8();
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          f32x4 e = {0.f, 0.f, 0.f, 0.f};
          e = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[sub][0], x0, e, 0, 0, 0);
          if (CinP > 32) e = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[sub][1], x1, e, 0, 0, 0);
          // lane holds hidden channels c0 + sub*16 + kq*4 + q of input pixel ip
          bf16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = fminf(fmaxf(e[q] + bias[sub][q], 0.f), 6.f);
            o[q] = (bf16)(inside ? v : 0.f);
          }
          *reinterpret_cast<bf16x4*>(E + (size_t)ip * ES + sub * 16 + kq * 4) = o;
        }
      }
      __syncthreads();
    }
    const bf16* src = EXPAND ? E : X + c0;
    const int sstride = EXPAND ? ES : XS;

    // ---- 2b. depthwise for this lane's 8 channels of its two output pixels
    // (both pixels per tap, so each tap's weights are loaded once and live briefly)
    const float4 b0 = *reinterpret_cast<const float4*>(a.bd + c0 + kq * 8);
    const float4 b1 = *reinterpret_cast<const float4*>(a.bd + c0 + kq * 8 + 4);
    float d[GPW][8];
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      d[g][0] = b0.x; d[g][1] = b0.y; d[g][2] = b0.z; d[g][3] = b0.w;
      d[g][4] = b1.x; d[g][5] = b1.y; d[g][6] = b1.z; d[g][7] = b1.w;
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int tap = ky * 3 + kx;
        const float4 w0 = *reinterpret_cast<const float4*>(a.wd + tap * a.hidP + c0 + kq * 8);
        const float4 w1 = *reinterpret_cast<const float4*>(a.wd + tap * a.hidP + c0 + kq * 8 + 4);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int g = 0; g < GPW; ++g) {
          const int ip = ((wid * GPW + g) * s + ky) * TIW + r16 * s + kx;
          const bf16x8 v = ld8(src + (size_t)ip * sstride + kq * 8);
#pragma unroll
          for (int q = 0; q < 8; ++q) d[g][q] += (float)v[q] * wv[q];
        }
      }
    bf16x8 dfrag[GPW];
#pragma unroll
    for (int g = 0; g < GPW; ++g)
#pragma unroll
      for (int q = 0; q < 8; ++q) dfrag[g][q] = (bf16)fminf(fmaxf(d[g][q], 0.f), 6.f);

    // ---- 2c. project chunk (MFMA), A = projection weights
#pragma unroll
    for (int n = 0; n < NSUB; ++n) {
      const bf16x8 af = ld8(a.wp + (size_t)(n * 16 + r16) * a.hidP + c0 + kq * 8);
#pragma unroll
      for (int g = 0; g < GPW; ++g)
        acc[g][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, dfrag[g], acc[g][n], 0, 0, 0);
    }
    if (EXPAND) __syncthreads();  // E is rewritten by the next chunk
  }

  // ---- 3. epilogue: lane holds out channels n*16 + kq*4 + q of pixel (ty, r16)
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    const int ty = wid * GPW + g, tx = r16;
    const int oy = oy0 + ty, ox = ox0 + tx;
    if (oy >= a.OH || ox >= a.OW) continue;
    bf16* op = a.out + (((long long)b * a.OH + oy) * a.OW + ox) * a.Cout;
    const bf16* rp = X + (size_t)((ty * s + 1) * TIW + tx * s + 1) * (a.CinP + 8);
#pragma unroll
    for (int n = 0; n < NSUB; ++n) {
      const int co = n * 16 + kq * 4;
      if (co >= a.Cout) continue;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = acc[g][n][q] + a.bp[co + q];
        if (a.residual) v[q] += (float)rp[co + q];
      }
      if (co + 3 < a.Cout && (a.Cout & 3) == 0) {
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)v[q];
        *reinterpret_cast<bf16x4*>(op + co) = o;
      } else {
        for (int q = 0; q < 4; ++q)
          if (co + q < a.Cout) op[co + q] = (bf16)v[q];
      }
    }
  }
}

template <int NSUB, bool EXPAND, int GPW>
void launch_ir(const IRArgs& a, hipStream_t st) {
  constexpr int TH = 4 * GPW;
  const int s = a.stride;
  const int in_px = ((TH - 1) * s + 3) * ((TW - 1) * s + 3);
  const int in_groups = (in_px + 15) / 16;
  const size_t lds = (size_t)in_groups * 16 * (a.CinP + 8 + (EXPAND ? 40 : 0)) * sizeof(bf16);
  const int grid = a.B * cdiv(a.OH, TH) * cdiv(a.OW, TW);
  static bool attr_set = false;  // > 64 KB of dynamic LDS needs the opt-in attribute
  if (!attr_set) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_ir_kernel<NSUB, EXPAND, GPW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "fused_ir attr");
    attr_set = true;
  }
  hipLaunchKernelGGL((fused_ir_kernel<NSUB, EXPAND, GPW>), dim3(grid), dim3(256), lds, st, a);
  check_launch("fused_ir");
}


// ---------------------------------------------------------------------------
// General 2-D tile variant (any stride/dilation, Cin <= 160, Cout <= 320, with or
// without expansion). Output pixel p of the tile is (p / TX, p % TX); 16-pixel
// MFMA groups are assigned GPW per wave, so the lane -> pixel map is arbitrary
// and the depthwise reads use per-lane LDS addresses. 33 = 3 x 11, so 11x11 /
// 5x11 tiles cover the 33x33 maps with no waste where 16-wide tiles waste 31 %.
//
// Internals run in fp16 (PMC: the bf16/fp32 version was VALU-bound — 2k VALU
// instructions per wave, ~45 % of the kernel — on bf16->f32 unpacking and scalar
// FMAs): the expansion epilogue writes relu6(x) as fp16 into LDS, the depthwise
// runs as v_pk_fma_f16 (2 MACs per instruction, no unpacking), and the projection
// uses v_mfma_f32_16x16x32_f16 on fp16 weights, so the depthwise result feeds the
// MFMA with no conversion. relu6-bounded activations lose nothing in fp16 (11-bit
// mantissa vs bf16's 8); accumulation of the projection stays fp32.
typedef _Float16 f16;
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct IRTArgs {
  const bf16* in; const bf16* we; const float* be; const f16* wd; const f16* bd;
  const f16* wp; const float* bp; bf16* out;
  int B, IH, IW, Cin, hidP, Cout, OH, OW, stride, dil, residual, TY, TX, tiles_y, tiles_x;
  long long* trace;  // debug: s_memtime stamps of workgroup 0 / wave 0 (null = off)
};

#define IR_STAMP(k)                                                                 \
  do {                                                                              \
    if (a.trace && blockIdx.x == 0 && threadIdx.x == 0) a.trace[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)

template <int NSUB, int KS, int GPW, bool EXPAND, int NW>
__global__ __launch_bounds__(64 * NW) void fused_ir_tile_kernel(IRTArgs a) {
  constexpr int NT = 64 * NW;  // threads
  constexpr int CinP = KS * 32;
  constexpr int XS = CinP + 8, ES = 32 + 8;  // +16 B per LDS row: conflict-free ds_read_b128
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = a.stride, dl = a.dil;
  const int TIH = (a.TY - 1) * s + 2 * dl + 1, TIW = (a.TX - 1) * s + 2 * dl + 1;
  const int in_px = TIH * TIW;
  const int in_groups = (in_px + 15) / 16;
  bf16* X = reinterpret_cast<bf16*>(smem);  // EXPAND only
  f16* E = reinterpret_cast<f16*>(smem + (EXPAND ? (size_t)in_groups * 16 * XS * sizeof(bf16) : 0));

  const int ntile = a.tiles_y * a.tiles_x;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring tiles share halos: same XCD L2
  const int b = bid / ntile, t = bid % ntile;
  const int oy0 = (t / a.tiles_x) * a.TY, ox0 = (t % a.tiles_x) * a.TX;
  const int iy0 = oy0 * s - dl, ix0 = ox0 * s - dl;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  IR_STAMP(0);
  // expansion weights are software-pipelined one chunk ahead: s_memtime timelines
  // showed every chunk's expansion stalled ~2.5k cycles on these loads (L2 under
  // load), longer than the chunk's MFMA + depthwise work
  bf16x8 wfr_n[2][KS];
  f32x4 bias_n[2];
  auto load_expand_w = [&](int c) {
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const bf16* wrow = a.we + (size_t)(c + sub * 16 + r16) * CinP;
#pragma unroll
      for (int k = 0; k < KS; ++k) wfr_n[sub][k] = ld8(wrow + k * 32 + kq * 8);
      bias_n[sub] = *reinterpret_cast<const f32x4*>(a.be + c + sub * 16 + kq * 4);
    }
  };
  if (EXPAND) load_expand_w(0);  // overlaps the input-tile staging

  if (EXPAND) {
    constexpr int cpp = CinP / 8;
    for (int i = tid; i < in_groups * 16 * cpp; i += NT) {
      const int ip = i / cpp, c = (i % cpp) * 8;
      const int ty = ip / TIW, tx = ip - ty * TIW;
      const int iy = iy0 + ty, ix = ix0 + tx;
      bf16x8 v = zero8();
      if (ip < in_px && c < a.Cin && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW)
        v = ld8(a.in + (((long long)b * a.IH + iy) * a.IW + ix) * a.Cin + c);
      st8(X + (size_t)ip * XS + c, v);
    }
  } else {  // depthwise straight on the input: stage it as fp16 (hidP == CinP == 32)
    for (int i = tid; i < in_groups * 16 * 4; i += NT) {
      const int ip = i >> 2, c = (i & 3) * 8;
      const int ty = ip / TIW, tx = ip - ty * TIW;
      const int iy = iy0 + ty, ix = ix0 + tx;
      f16x8 h = {0, 0, 0, 0, 0, 0, 0, 0};
      if (ip < in_px && c < a.Cin && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW) {
        const bf16x8 v = ld8(a.in + (((long long)b * a.IH + iy) * a.IW + ix) * a.Cin + c);
#pragma unroll
        for (int q = 0; q < 8; ++q) h[q] = (f16)(float)v[q];
      }
      *reinterpret_cast<f16x8*>(E + (size_t)ip * ES + c) = h;
    }
  }

  int pofs[GPW], oyv[GPW], oxv[GPW];
  bool pval[GPW];
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    const int p = (wid * GPW + g) * 16 + r16;
    const int py = p / a.TX, px = p - py * a.TX;
    oyv[g] = oy0 + py;
    oxv[g] = ox0 + px;
    pval[g] = p < a.TY * a.TX && oyv[g] < a.OH && oxv[g] < a.OW;
    pofs[g] = pval[g] ? (py * s) * TIW + px * s : 0;
  }
  __syncthreads();

  IR_STAMP(1);
  f32x4 acc[GPW][NSUB];
#pragma unroll
  for (int g = 0; g < GPW; ++g)
#pragma unroll
    for (int n = 0; n < NSUB; ++n) acc[g][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f16x8 h0 = {0, 0, 0, 0, 0, 0, 0, 0}, h6 = {6, 6, 6, 6, 6, 6, 6, 6};


  for (int c0 = 0; c0 < a.hidP; c0 += 32) {
    // this chunk's depthwise / projection weights: issued first, in flight under the expansion
    f16x8 wdv[9];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
      wdv[tap] = *reinterpret_cast<const f16x8*>(a.wd + tap * a.hidP + c0 + kq * 8);
    const f16x8 bdv = *reinterpret_cast<const f16x8*>(a.bd + c0 + kq * 8);
    f16x8 af[NSUB];
#pragma unroll
    for (int n = 0; n < NSUB; ++n)
      af[n] = *reinterpret_cast<const f16x8*>(a.wp + (size_t)(n * 16 + r16) * a.hidP + c0 + kq * 8);

    if (EXPAND) {
      bf16x8 wfr[2][KS];
      f32x4 bias[2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
        for (int k = 0; k < KS; ++k) wfr[sub][k] = wfr_n[sub][k];
        bias[sub] = bias_n[sub];
      }
      for (int gi = wid; gi < in_groups; gi += NW) {
        const int ip = gi * 16 + r16;
        const int ty = ip / TIW, tx = ip - ty * TIW;
        const int iy = iy0 + ty, ix = ix0 + tx;
        const bool inside = ip < in_px && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
        bf16x8 xf[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k) xf[k] = ld8(X + (size_t)ip * XS + k * 32 + kq * 8);
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          f32x4 e = bias[sub];
#pragma unroll
          for (int k = 0; k < KS; ++k)
            e = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[sub][k], xf[k], e, 0, 0, 0);
          f16x4 o = {(f16)e[0], (f16)e[1], (f16)e[2], (f16)e[3]};
          o = __builtin_elementwise_min(__builtin_elementwise_max(o, h0.lo), h6.lo);
          if (!inside) o = h0.lo;  // zero padding applies to the expanded tensor
          *reinterpret_cast<f16x4*>(E + (size_t)ip * ES + sub * 16 + kq * 4) = o;
        }
      }
      IR_STAMP(2 + 4 * (c0 / 32));
      __syncthreads();
      IR_STAMP(3 + 4 * (c0 / 32));
      if (c0 + 32 < a.hidP) load_expand_w(c0 + 32);  // in flight under depthwise + projection
    }

    // ---- depthwise (packed fp16): lane -> 8 channels (kq*8..) of its pixel in each group
    f16x8 d[GPW];
#pragma unroll
    for (int g = 0; g < GPW; ++g) d[g] = bdv;
    // all taps' LDS reads first, then the FMAs: with one or two waves per SIMD a
    // read-use-read chain exposes the LDS latency on every tap
    f16x8 v[GPW][9];
#pragma unroll
    for (int g = 0; g < GPW; ++g)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
        v[g][tap] = *reinterpret_cast<const f16x8*>(
            E + (size_t)(pofs[g] + ((tap / 3) * TIW + tap % 3) * dl) * ES + kq * 8);
#pragma unroll
    for (int g = 0; g < GPW; ++g)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) d[g] = v[g][tap] * wdv[tap] + d[g];
#pragma unroll
    for (int g = 0; g < GPW; ++g) d[g] = __builtin_elementwise_min(__builtin_elementwise_max(d[g], h0), h6);

    IR_STAMP(4 + 4 * (c0 / 32));
    // ---- project chunk (fp16 MFMA, fp32 accumulate)
#pragma unroll
    for (int n = 0; n < NSUB; ++n)
#pragma unroll
      for (int g = 0; g < GPW; ++g)
        acc[g][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[n], d[g], acc[g][n], 0, 0, 0);
    IR_STAMP(5 + 4 * (c0 / 32));
    if (EXPAND) __syncthreads();  // E is rewritten by the next chunk
  }
  IR_STAMP(126);

#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    if (!pval[g]) continue;
    bf16* op = a.out + (((long long)b * a.OH + oyv[g]) * a.OW + oxv[g]) * a.Cout;
    const bf16* rp = X + (size_t)(pofs[g] + dl * TIW + dl) * XS;
#pragma unroll
    for (int n = 0; n < NSUB; ++n) {
      const int co = n * 16 + kq * 4;
      if (co >= a.Cout) continue;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = acc[g][n][q] + a.bp[co + q];
        if (EXPAND && a.residual) v[q] += (float)rp[co + q];
      }
      if (co + 3 < a.Cout && (a.Cout & 3) == 0) {
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)v[q];
        *reinterpret_cast<bf16x4*>(op + co) = o;
      } else {
        for (int q = 0; q < 4; ++q)
          if (co + q < a.Cout) op[co + q] = (bf16)v[q];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Stem + first inverted residual in one kernel (MobileNetV2 blocks 0: no
// expansion, dw 3x3 on the 32 stem channels, project 32 -> 16). The 257^2 x 32
// stem activation (135 MB per 32 frames) is the largest tensor of the network and
// this fusion never writes it: per TY x TX output tile, the letterboxed camera
// pixels under the tile's receptive field are gathered through the LUTs into LDS
// (normalised, bf16), the stem conv runs on MFMA (K = 3x3x3 = 27 padded to 32:
// one v_mfma_f32_16x16x32_bf16 per 16 pixels x 16 channels) over the tile plus its
// 1-pixel halo, relu6 in fp16 into LDS, then the tile kernel's packed-fp16
// depthwise and fp16-MFMA projection.
struct SB0Args {
  const uint8_t* frames; const int32_t* lut_x; const int32_t* lut_y;
  const bf16* ws;  // stem weights [32 out][48 K] bf16, K = tap*4 + c (RGB + zero), taps 9..11 zero
  const float* bs; // stem bias [32]
  const f16* wd; const f16* bd;  // depthwise [9][32], [32] fp16
  const f16* wp;   // projection [16][32] fp16
  const float* bp; // [16]
  bf16* out;       // [B, SH, SW, Cout]
  int B, Hc, Wc, H, W, SH, SW, Cout, TY, TX, tiles_y, tiles_x;
};

typedef short s16x4 __attribute__((ext_vector_type(4)));

// i / d for the small non-negative tile indices here (i < 2^14, d < 128): one
// float multiply instead of a ~20-instruction integer division (the kernel is
// VALU-bound; these divisions were a large share of its instructions)
__device__ __forceinline__ int sdiv(int i, float inv_d) { return (int)(((float)i + 0.5f) * inv_d); }

template <int GPW>
__global__ __launch_bounds__(256) void stem_block0_kernel(SB0Args a) {
  constexpr int ES = 32 + 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int SHT = a.TY + 2, SWT = a.TX + 2;        // stem tile incl. halo
  const int IHT = 2 * SHT + 1, IWT = 2 * SWT + 1;  // model-input region
  const int s_px = SHT * SWT, s_groups = (s_px + 15) / 16;
  bf16* IN = reinterpret_cast<bf16*>(smem);                                   // [IHT*IWT][4]
  f16* E = reinterpret_cast<f16*>(smem + ((size_t)IHT * IWT * 8 + 15) / 16 * 16);  // [s_groups*16][ES]
  const int ntile = a.tiles_y * a.tiles_x;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bid / ntile, t = bid % ntile;
  const int oy0 = (t / a.tiles_x) * a.TY, ox0 = (t % a.tiles_x) * a.TX;
  const int sy0 = oy0 - 1, sx0 = ox0 - 1;           // stem tile origin
  const int iy0 = 2 * sy0 - 1, ix0 = 2 * sx0 - 1;   // input region origin
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const float inv_swt = 1.f / SWT, inv_tx = 1.f / a.TX;

  const uint8_t* fb = a.frames + (size_t)b * a.Hc * a.Wc * 3;
  gather_letterbox_rgb0<6, 256>(IN, fb, a.lut_x, a.lut_y, a.Wc, a.H, a.W, iy0, ix0, IHT, IWT, tid);
  // Stem conv on v_mfma_f32_16x16x16_bf16: K = 12 taps x 4 channels (RGB + the zero
  // 4th channel of IN, taps 9..11 zero) in 3 MFMAs; lane kq of MFMA m holds tap
  // 4m + kq, i.e. ONE 8-byte LDS read of the pixel's 4 channels (no per-element
  // gathers). A operand: weight rows sub*16 + r16, K = m*16 + kq*4 .. +3.
  s16x4 wst[2][3];
  f32x4 bst[2];
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
    for (int m = 0; m < 3; ++m)
      wst[sub][m] = *reinterpret_cast<const s16x4*>(a.ws + (size_t)(sub * 16 + r16) * 48 + m * 16 + kq * 4);
    bst[sub] = *reinterpret_cast<const f32x4*>(a.bs + sub * 16 + kq * 4);
  }
  int toff[3];  // element offset of this lane's tap in IN, relative to the window origin
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int tp = m * 4 + kq;
    toff[m] = tp < 9 ? ((tp / 3) * IWT + tp % 3) * 4 : -1;
  }
  __syncthreads();
  // ReLU6 as a [0, 1] clamp (ops/hip_ops.pack_stem_block0 packs the stem / 6, the depthwise
  // bias / 6 and the projection x 6): the clamps fold into the conversion / the last fma
  const f16x4 z4 = {0, 0, 0, 0}, s4 = {1, 1, 1, 1};
  const s16x4 zs = {0, 0, 0, 0};
  for (int gi = wid; gi < s_groups; gi += 4) {
    const int sp = gi * 16 + r16;
    const int ty = sdiv(sp, inv_swt), tx = sp - ty * SWT;
    const int sy = sy0 + ty, sx = sx0 + tx;
    const bool inside = sp < s_px && sy >= 0 && sy < a.SH && sx >= 0 && sx < a.SW;
    const int base = sp < s_px ? ((2 * ty) * IWT + 2 * tx) * 4 : 0;
    s16x4 xf[3];
#pragma unroll
    for (int m = 0; m < 3; ++m)
      xf[m] = toff[m] >= 0 ? *reinterpret_cast<const s16x4*>(IN + base + toff[m]) : zs;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x4 e4 = bst[sub];
#pragma unroll
      for (int m = 0; m < 3; ++m) e4 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wst[sub][m], xf[m], e4, 0, 0, 0);
      f16x4 o = {(f16)e4[0], (f16)e4[1], (f16)e4[2], (f16)e4[3]};
      o = __builtin_elementwise_min(__builtin_elementwise_max(o, z4), s4);
      if (!inside) o = z4;  // depthwise zero padding outside the stem image
      *reinterpret_cast<f16x4*>(E + (size_t)sp * ES + sub * 16 + kq * 4) = o;
    }
  }
  // depthwise / projection weights
  f16x8 wdv[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) wdv[tap] = *reinterpret_cast<const f16x8*>(a.wd + tap * 32 + kq * 8);
  const f16x8 bdv = *reinterpret_cast<const f16x8*>(a.bd + kq * 8);
  const f16x8 af = *reinterpret_cast<const f16x8*>(a.wp + (size_t)r16 * 32 + kq * 8);
  __syncthreads();
  const f16x8 h0 = {0, 0, 0, 0, 0, 0, 0, 0}, h6 = {1, 1, 1, 1, 1, 1, 1, 1};  // [0, 1]: see s4
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    const int p = (wid * GPW + g) * 16 + r16;
    const int py = sdiv(p, inv_tx), px = p - py * a.TX;
    const int oy = oy0 + py, ox = ox0 + px;
    const bool valid = p < a.TY * a.TX && oy < a.SH && ox < a.SW;
    const int pofs = valid ? py * SWT + px : 0;
    f16x8 v[9];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
      v[tap] = *reinterpret_cast<const f16x8*>(E + (size_t)(pofs + (tap / 3) * SWT + tap % 3) * ES + kq * 8);
    f16x8 d = bdv;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) d = v[tap] * wdv[tap] + d;
    d = __builtin_elementwise_min(__builtin_elementwise_max(d, h0), h6);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, d, acc, 0, 0, 0);
    if (!valid) continue;
    const int co = kq * 4;
    if (co >= a.Cout) continue;
    bf16* op = a.out + (((size_t)b * a.SH + oy) * a.SW + ox) * a.Cout + co;
    bf16x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = (bf16)(acc[q] + a.bp[co + q]);
    *reinterpret_cast<bf16x4*>(op) = o;
  }
}

size_t tile_lds_bytes(int CinP, int stride, int dil, int TY, int TX, bool expand = true) {
  const int in_px = ((TY - 1) * stride + 2 * dil + 1) * ((TX - 1) * stride + 2 * dil + 1);
  return (size_t)((in_px + 15) / 16) * 16 * ((expand ? CinP + 8 : 0) + 40) * 2;
}

template <int NSUB, int KS, int GPW, bool EX, int NW>
void launch_ir_tile_nw(const IRTArgs& a, size_t lds, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_ir_tile_kernel<NSUB, KS, GPW, EX, NW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "fused_ir_tile attr");
    attr_set = true;
  }
  const int grid = a.B * a.tiles_y * a.tiles_x;
  hipLaunchKernelGGL((fused_ir_tile_kernel<NSUB, KS, GPW, EX, NW>), dim3(grid), dim3(64 * NW), lds, st, a);
  check_launch("fused_ir_tile");
}

// groups = ceil(TY*TX / 16) pixel groups: 4 waves x GPW (GPW 1/2)
template <int NSUB, int KS, bool EX>
void launch_ir_tile(const IRTArgs& a, int groups, size_t lds, hipStream_t st) {
  // (8 waves x 1 group measured 1.3-2x slower than 4 x 2 on every 33x33 block)
  if (groups <= 4) launch_ir_tile_nw<NSUB, KS, 1, EX, 4>(a, lds, st);
  else launch_ir_tile_nw<NSUB, KS, 2, EX, 4>(a, lds, st);
}

void fused_ir_tile(const FusedIRParams& p, hipStream_t st) {
  if (!p.wd_h || !p.bd_h || !p.wp_h) throw std::invalid_argument("fused_ir_tile: needs the fp16 weights");
  if (p.dil < 1 || p.TX < 1 || p.TY < 1) throw std::invalid_argument("fused_ir_tile: bad tile");
  if (p.Cin % 8 || p.hidP % 32 || p.CinP % 32 || p.CinP < p.Cin)
    throw std::invalid_argument("fused_ir_tile: bad channel padding");
  const bool ex = p.we != nullptr;
  if (!ex && (p.CinP != 32 || p.hidP != 32 || p.residual))
    throw std::invalid_argument("fused_ir_tile: no-expansion blocks need Cin <= 32 and no residual");
  if (p.residual && (p.stride != 1 || p.Cin != p.Cout)) throw std::invalid_argument("fused_ir_tile: bad residual");
  const int groups = (p.TY * p.TX + 15) / 16;
  const int gpw = (groups + 3) / 4;
  const size_t lds = tile_lds_bytes(p.CinP, p.stride, p.dil, p.TY, p.TX, ex);
  if (gpw > 2 || lds > 160 * 1024) throw std::invalid_argument("fused_ir_tile: tile too large");
  IRTArgs a{p.in, p.we, p.be, reinterpret_cast<const f16*>(p.wd_h), reinterpret_cast<const f16*>(p.bd_h),
            reinterpret_cast<const f16*>(p.wp_h), p.bp, p.out, p.B, p.IH, p.IW, p.Cin, p.hidP,
            p.Cout, p.OH, p.OW, p.stride, p.dil, p.residual, p.TY, p.TX,
            cdiv(p.OH, p.TY), cdiv(p.OW, p.TX), p.trace};
  const int nsub = (p.Cout + 15) / 16, ks = p.CinP / 32;
  if (!ex) {
    if (nsub == 1) {
      launch_ir_tile<1, 1, false>(a, groups, lds, st);
      return;
    }
    throw std::invalid_argument("fused_ir_tile: unsupported no-expansion Cout");
  }
#define IRT(N, K)                                                        \
  if (nsub == N && ks == K) {                                            \
    launch_ir_tile<N, K, true>(a, groups, lds, st);                      \
    return;                                                              \
  }
  IRT(4, 2) IRT(6, 2) IRT(6, 3) IRT(10, 3) IRT(10, 5) IRT(20, 5) IRT(4, 1) IRT(2, 1)
#undef IRT
  throw std::invalid_argument("fused_ir_tile: unsupported (Cout, Cin) combination");
}

}  // namespace

void stem_block0(const StemBlock0Params& p, hipStream_t st) {
  if (p.Cout != 16) throw std::invalid_argument("stem_block0: block 0 must project to 16 channels");
  if (p.TY < 1 || p.TX < 1 || (p.TY * p.TX + 15) / 16 > 16 || p.TX > 120)
    throw std::invalid_argument("stem_block0: bad tile");
  if (p.SH != (p.H - 1) / 2 + 1 || p.SW != (p.W - 1) / 2 + 1) throw std::invalid_argument("stem_block0: bad stem size");
  SB0Args a{p.frames, p.lut_x, p.lut_y, p.ws, p.bs, reinterpret_cast<const f16*>(p.wd),
            reinterpret_cast<const f16*>(p.bd), reinterpret_cast<const f16*>(p.wp), p.bp, p.out,
            p.B, p.Hc, p.Wc, p.H, p.W, p.SH, p.SW, p.Cout, p.TY, p.TX, cdiv(p.SH, p.TY), cdiv(p.SW, p.TX)};
  const int SHT = p.TY + 2, SWT = p.TX + 2;
  const size_t lds = ((size_t)(2 * SHT + 1) * (2 * SWT + 1) * 8 + 15) / 16 * 16 +
                     (size_t)((SHT * SWT + 15) / 16) * 16 * 40 * 2;
  const int grid = p.B * a.tiles_y * a.tiles_x;
  const int groups = (p.TY * p.TX + 15) / 16;
  if (lds > 160 * 1024) throw std::invalid_argument("stem_block0: tile too large for LDS");
  static bool attr = false;
  if (!attr) {
    for (const void* k : {reinterpret_cast<const void*>(&stem_block0_kernel<1>),
                          reinterpret_cast<const void*>(&stem_block0_kernel<2>),
                          reinterpret_cast<const void*>(&stem_block0_kernel<4>)})
      check(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024), "stem_block0 attr");
    attr = true;
  }
  if (groups <= 4)
    hipLaunchKernelGGL(stem_block0_kernel<1>, dim3(grid), dim3(256), lds, st, a);
  else if (groups <= 8)
    hipLaunchKernelGGL(stem_block0_kernel<2>, dim3(grid), dim3(256), lds, st, a);
  else
    hipLaunchKernelGGL(stem_block0_kernel<4>, dim3(grid), dim3(256), lds, st, a);
  check_launch("stem_block0");
}

size_t fused_ir_tile_lds(int CinP, int stride, int dil, int TY, int TX, int expand) {
  return tile_lds_bytes(CinP, stride, dil, TY, TX, expand != 0);
}

void fused_inverted_residual(const FusedIRParams& p, hipStream_t st) {
  if (p.TY > 0) {
    fused_ir_tile(p, st);
    return;
  }
  if (p.stride != 1 && p.stride != 2) throw std::invalid_argument("fused_ir: stride must be 1 or 2");
  if (p.CinP % 32 || p.hidP % 32 || p.CinP < p.Cin || p.CinP > 64)
    throw std::invalid_argument("fused_ir: CinP must be 32 or 64 and >= Cin");
  if (p.residual && (p.stride != 1 || p.Cin != p.Cout)) throw std::invalid_argument("fused_ir: bad residual");
  if (p.Cin % 8) throw std::invalid_argument("fused_ir: Cin must be a multiple of 8");
  IRArgs a{p.in, p.we, p.be, p.wd, p.bd, p.wp, p.bp, p.out, p.B, p.IH, p.IW, p.Cin, p.CinP,
           p.hidP, p.Cout, p.OH, p.OW, p.stride, p.residual};
  const int nsub = (p.Cout + 15) / 16;
  const bool ex = p.we != nullptr;
  if (!ex && p.hidP != p.CinP) throw std::invalid_argument("fused_ir: no-expand needs hidP == CinP");
  // stride 2: 4-row tiles (9 x 33 input tile, ~49 KB LDS, 3 workgroups/CU);
  // stride 1: 8-row tiles (10 x 18 input tile)
#define IR_CASE(N)                                                   \
  case N:                                                            \
    if (p.stride == 2) {                                             \
      if (ex) launch_ir<N, true, 1>(a, st);                          \
      else launch_ir<N, false, 1>(a, st);                            \
    } else {                                                         \
      if (ex) launch_ir<N, true, 2>(a, st);                          \
      else launch_ir<N, false, 2>(a, st);                            \
    }                                                                \
    break;
  switch (nsub) {
    IR_CASE(1)
    IR_CASE(2)
    IR_CASE(3)
    IR_CASE(4)
    IR_CASE(6)
    default:
      throw std::invalid_argument("fused_ir: unsupported Cout");
  }
#undef IR_CASE
}

namespace {

// ---------------------------------------------------------------------------
// Depthwise + projection fusion for the low-resolution, wide blocks (33x33 maps,
// hid 384..960, dilation 1/2) where full fusion would recompute the expansion
// over large halos: the expanded tensor comes from the MFMA GEMM as usual, but the
// depthwise result never leaves registers — each lane's 8 depthwise channels of
// one pixel are its B fragment for the projection MFMA.
// Workgroup: 64 consecutive output pixels (4 waves x 16) x one slice of NSUB*16
// output channels (blockIdx.y); K loop over the hidden channels in 32-chunks.
struct DPArgs {
  const bf16* hid_in;  // [B, IH, IW, hid] expanded activations
  const float* wd;     // [9, hid]
  const float* bd;     // [hid]
  const bf16* wp;      // [CoutP, hid]
  const float* bp;     // [CoutP]
  const bf16* res;     // optional [B, OH, OW, Cout]
  bf16* out;           // [B, OH, OW, Cout]
  int B, IH, IW, hid, Cout, OH, OW, stride, dil;
};

template <int NSUB>
__global__ __launch_bounds__(256) void dw_project_kernel(DPArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int M = a.B * a.OH * a.OW;
  const int m = blockIdx.x * 64 + wid * 16 + r16;
  const bool valid = m < M;
  const int mm = valid ? m : 0;
  const int b = mm / (a.OH * a.OW);
  const int rem = mm - b * a.OH * a.OW;
  const int oy = rem / a.OW, ox = rem % a.OW;
  const int n0 = blockIdx.y * NSUB * 16;
  long long off[9];
  bool ok[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int iy = oy * a.stride + (t / 3 - 1) * a.dil, ix = ox * a.stride + (t % 3 - 1) * a.dil;
    ok[t] = valid && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
    off[t] = (((long long)b * a.IH + iy) * a.IW + ix) * a.hid;
  }
  f32x4 acc[NSUB];
#pragma unroll
  for (int n = 0; n < NSUB; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < a.hid; c0 += 32) {
    const int c = c0 + kq * 8;
    bf16x8 v[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) v[t] = ok[t] ? ld8(a.hid_in + off[t] + c) : zero8();
    const float4 b0 = *reinterpret_cast<const float4*>(a.bd + c);
    const float4 b1 = *reinterpret_cast<const float4*>(a.bd + c + 4);
    float d[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 w0 = *reinterpret_cast<const float4*>(a.wd + t * a.hid + c);
      const float4 w1 = *reinterpret_cast<const float4*>(a.wd + t * a.hid + c + 4);
      d[0] += (float)v[t][0] * w0.x; d[1] += (float)v[t][1] * w0.y;
      d[2] += (float)v[t][2] * w0.z; d[3] += (float)v[t][3] * w0.w;
      d[4] += (float)v[t][4] * w1.x; d[5] += (float)v[t][5] * w1.y;
      d[6] += (float)v[t][6] * w1.z; d[7] += (float)v[t][7] * w1.w;
    }
    bf16x8 df;
#pragma unroll
    for (int q = 0; q < 8; ++q) df[q] = (bf16)fminf(fmaxf(d[q], 0.f), 6.f);
#pragma unroll
    for (int n = 0; n < NSUB; ++n) {
      const bf16x8 af = ld8(a.wp + (size_t)(n0 + n * 16 + r16) * a.hid + c);
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, df, acc[n], 0, 0, 0);
    }
  }
  if (!valid) return;
  bf16* op = a.out + (long long)mm * a.Cout;
#pragma unroll
  for (int n = 0; n < NSUB; ++n) {
    const int co = n0 + n * 16 + kq * 4;
    if (co >= a.Cout) continue;
    float vv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      vv[q] = acc[n][q] + a.bp[co + q];
      if (a.res && co + q < a.Cout) vv[q] += (float)a.res[(long long)mm * a.Cout + co + q];
    }
    if (co + 3 < a.Cout && (a.Cout & 3) == 0) {
      bf16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = (bf16)vv[q];
      *reinterpret_cast<bf16x4*>(op + co) = o;
    } else {
      for (int q = 0; q < 4; ++q)
        if (co + q < a.Cout) op[co + q] = (bf16)vv[q];
    }
  }
}

}  // namespace (dw_project)

void dw_project(const DwProjectParams& p, hipStream_t st) {
  if (p.hid % 32) throw std::invalid_argument("dw_project: hid must be a multiple of 32");
  DPArgs a{p.hid_in, p.wd, p.bd, p.wp, p.bp, p.res, p.out, p.B, p.IH, p.IW, p.hid, p.Cout,
           p.OH, p.OW, p.stride, p.dil};
  const int M = p.B * p.OH * p.OW;
  const int nsub_total = (p.Cout + 15) / 16;
  // channel slices of up to 5 subtiles (80 channels): more workgroups, fewer VGPRs
  int nsub = nsub_total;
  for (int cand : {5, 4, 3, 2, 1})
    if (nsub_total % cand == 0 && nsub_total / cand <= 4) { nsub = cand; break; }
  if (nsub_total <= 6) nsub = nsub_total;
  const dim3 grid(cdiv(M, 64), nsub_total / nsub);
#define DP_CASE(N) \
  case N: hipLaunchKernelGGL(dw_project_kernel<N>, grid, dim3(256), 0, st, a); break;
  switch (nsub) {
    DP_CASE(1) DP_CASE(2) DP_CASE(3) DP_CASE(4) DP_CASE(5) DP_CASE(6)
    default: throw std::invalid_argument("dw_project: unsupported Cout");
  }
#undef DP_CASE
  check_launch("dw_project");
}

namespace {  // reopen for nothing (keeps the file's namespace structure simple)
}  // namespace

}  // namespace ssa
