// int8 implicit-GEMM convolution on the CDNA4 int8 MFMA (v_mfma_i32_16x16x64_i8),
// NHWC int8 activations (per-tensor symmetric scale), int8 weights (per output
// channel), exact int32 accumulation, fused epilogue:
//
//   v = acc * scale[n] + bias[n] + img_bias[b][n] + res_i8 * res_scale
//   v = act(v);  out = out_mode == I8 ? clamp(round(v * inv_out_scale)) : bf16(v)
//
// scale[n] = in_scale * w_scale[n] is folded on the host. Used by the int8
// DeepLabv3-ResNet50 config (bottleneck 1x1/3x3 incl. strided, ASPP branches into
// a shared-scale concat buffer, projection, and the bf16-output logits layer).
// Mapping mirrors conv_gemm: A = weights (rows = out channels), B = pixels, so a
// lane's accumulator holds 4 consecutive output channels of one pixel; each
// fragment is one 16-byte load of 16 consecutive K elements
// (lane l: row/col l&15, k = 16*(l>>4) .. +15).
#include "common.h"
#include "kernels.h"

namespace ssa {
namespace {

typedef int i32x4v __attribute__((ext_vector_type(4)));

struct I8Args {
  const int8_t* in; const int8_t* w; const float* scale; const float* bias;
  const float* img_bias; const int8_t* res; float res_scale; void* out; float inv_out_scale;
  int out_mode;  // 0 int8, 1 bf16
  int B, IH, IW, Cin, OH, OW, Cout, KH, KW, stride, dil, ldo, co_off, act;
  const int* perm;  // LDS-DMA kernels: GEMM row -> output pixel, -1 = padding (tap-class tiles)
  int Mp;           // rows of perm
  int nmajor;       // LDS-DMA tile order: 0 row-major (m-tile, n-tile), 1 n-tile major (the
                    // dispatcher's consecutive blocks -> one XCD share one channel tile's weights)
};

__device__ __forceinline__ i32x4v ld16(const int8_t* p) { return *reinterpret_cast<const i32x4v*>(p); }

// int8 requantisation of 16 consecutive channels (n..n+15) of pixel m, folded into the
// affine terms: z = acc * (scale * ios) + (bias * ios + 128) + u * (res_scale * ios), u =
// residual byte + 128 (v_cvt_f32_ubyte on the XOR-ed word, the -128 folded into the bias);
// the activation and the int8 range are one med3 on the +128 offset grid, v_cvt_pk_u8_f32
// rounds (nearest even) and packs, XOR 0x80 gives the signed bytes. ~8 VALU per value
// instead of ~13 for the float chain, and within one rounding step of it (round 5).
// the 16 channels' folded constants: s = scale * ios, b = bias * ios + 128 - 128 * rs
struct I8Fold16 {
  float s[16], b[16];
};
__device__ __forceinline__ I8Fold16 i8_fold16(const I8Args& a, int n) {
  const float ios = a.inv_out_scale;
  const float rs = a.res ? a.res_scale * ios : 0.f;
  I8Fold16 f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float4 sc = *reinterpret_cast<const float4*>(a.scale + n + c * 4);
    const float4 bi = *reinterpret_cast<const float4*>(a.bias + n + c * 4);
    f.s[c * 4 + 0] = sc.x * ios; f.s[c * 4 + 1] = sc.y * ios; f.s[c * 4 + 2] = sc.z * ios; f.s[c * 4 + 3] = sc.w * ios;
    f.b[c * 4 + 0] = fmaf(bi.x, ios, 128.f - 128.f * rs); f.b[c * 4 + 1] = fmaf(bi.y, ios, 128.f - 128.f * rs);
    f.b[c * 4 + 2] = fmaf(bi.z, ios, 128.f - 128.f * rs); f.b[c * 4 + 3] = fmaf(bi.w, ios, 128.f - 128.f * rs);
  }
  return f;
}

__device__ __forceinline__ i32x4v i8_requant16(const I8Args& a, const i32x4v (&v)[4], int m, int n,
                                               const I8Fold16& f) {
  const float ios = a.inv_out_scale;
  const float rs = a.res ? a.res_scale * ios : 0.f;
  const float lo = a.act == ACT_NONE ? 1.f : 128.f;
  const float hi = a.act == ACT_RELU6 ? fminf(255.f, 128.f + 6.f * ios) : 255.f;
  unsigned ur[4] = {0, 0, 0, 0};
  if (a.res) {
    const i32x4v rv = *reinterpret_cast<const i32x4v*>(a.res + (size_t)m * a.Cout + n);
#pragma unroll
    for (int c = 0; c < 4; ++c) ur[c] = (unsigned)rv[c] ^ 0x80808080u;
  }
  i32x4v pk;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float s4[4] = {f.s[c * 4], f.s[c * 4 + 1], f.s[c * 4 + 2], f.s[c * 4 + 3]};
    float b4[4] = {f.b[c * 4], f.b[c * 4 + 1], f.b[c * 4 + 2], f.b[c * 4 + 3]};
    if (a.img_bias) {
      const int b = m / (a.OH * a.OW);
      const float4 ib = *reinterpret_cast<const float4*>(a.img_bias + (size_t)b * a.Cout + n + c * 4);
      b4[0] = fmaf(ib.x, ios, b4[0]); b4[1] = fmaf(ib.y, ios, b4[1]);
      b4[2] = fmaf(ib.z, ios, b4[2]); b4[3] = fmaf(ib.w, ios, b4[3]);
    }
    unsigned w = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float z = fmaf((float)v[c][q], s4[q], b4[q]);
      if (a.res) z = fmaf((float)((ur[c] >> (8 * q)) & 0xffu), rs, z);
      z = __builtin_amdgcn_fmed3f(z, lo, hi);
      w = __builtin_amdgcn_cvt_pk_u8_f32(z, q, w);
    }
    pk[c] = (int)(w ^ 0x80808080u);
  }
  return pk;
}

__device__ __forceinline__ i32x4v i8_requant16(const I8Args& a, const i32x4v (&v)[4], int m, int n) {
  return i8_requant16(a, v, m, n, i8_fold16(a, n));
}

// Transposing epilogue (NT == 4: a wave's 64 output channels): the MFMA C layout
// gives a lane 4 channels of one pixel per 16-channel subtile, so a direct store is
// 4 bytes per lane at a Cout stride and the int8 residual is read byte by byte.
// Per 16-pixel group the wave stages its int32 accumulators in LDS ([16 px][64 ch],
// 272-byte row pitch: both the writes and the reads hit 16 distinct bank groups per
// 16 lanes), reads them back as [pixel][16 consecutive channels] per lane and runs
// the epilogue on 16-byte vectors: float4 scale / bias, one 16-byte residual load,
// one 16-byte int8 (or 2 x 16-byte bf16) store.
constexpr int kEpPitch = 68;  // ints per staged pixel row (64 + 4 pad)

template <int MT>
__device__ __forceinline__ void i8_epilogue_lds(const I8Args& a, const i32x4v (&acc)[MT][4],
                                                int mbase, int nbase, int* ep, int lane) {
  const int M = a.B * a.OH * a.OW;
  const int r16 = lane & 15, kq = lane >> 4;
  const int px = lane >> 2, cb = (lane & 3) * 16;
  // the lane's 16 channels are the same for every pixel group: fold their constants once
  const bool fast = (a.Cout & 15) == 0 && a.out_mode == 0 && ((a.ldo | a.co_off) & 15) == 0;
  I8Fold16 fold;
  if (fast && nbase + cb + 16 <= a.Cout) fold = i8_fold16(a, nbase + cb);
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<i32x4v*>(ep + r16 * kEpPitch + j * 16 + kq * 4) = acc[i][j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    i32x4v v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = *reinterpret_cast<const i32x4v*>(ep + px * kEpPitch + cb + c * 4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the next group rewrites ep
    int m = mbase + i * 16 + px;
    const int n = nbase + cb;
    if (m >= (a.perm ? a.Mp : M) || n >= a.Cout) continue;
    if (a.perm && (m = a.perm[m]) < 0) continue;
    const int b = m / (a.OH * a.OW);
    float f[16];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) f[c * 4 + q] = (float)v[c][q];
    if (fast && n + 16 <= a.Cout) {
      *reinterpret_cast<i32x4v*>(static_cast<int8_t*>(a.out) + (size_t)m * a.ldo + a.co_off + n) =
          i8_requant16(a, v, m, n, fold);
    } else if (n + 16 <= a.Cout && (a.Cout & 15) == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 sc = *reinterpret_cast<const float4*>(a.scale + n + c * 4);
        const float4 bi = *reinterpret_cast<const float4*>(a.bias + n + c * 4);
        f[c * 4 + 0] = f[c * 4 + 0] * sc.x + bi.x; f[c * 4 + 1] = f[c * 4 + 1] * sc.y + bi.y;
        f[c * 4 + 2] = f[c * 4 + 2] * sc.z + bi.z; f[c * 4 + 3] = f[c * 4 + 3] * sc.w + bi.w;
        if (a.img_bias) {
          const float4 ib = *reinterpret_cast<const float4*>(a.img_bias + (size_t)b * a.Cout + n + c * 4);
          f[c * 4 + 0] += ib.x; f[c * 4 + 1] += ib.y; f[c * 4 + 2] += ib.z; f[c * 4 + 3] += ib.w;
        }
      }
      if (a.res) {
        const i32x4v rv = *reinterpret_cast<const i32x4v*>(a.res + (size_t)m * a.Cout + n);
        const signed char* rb = reinterpret_cast<const signed char*>(&rv);
#pragma unroll
        for (int q = 0; q < 16; ++q) f[q] += (float)rb[q] * a.res_scale;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) f[q] = apply_act(f[q], a.act);
      const size_t o = (size_t)m * a.ldo + a.co_off + n;
      if (a.out_mode == 0) {
        i32x4v pk;
        signed char* pb = reinterpret_cast<signed char*>(&pk);
#pragma unroll
        for (int q = 0; q < 16; ++q)
          pb[q] = (signed char)fminf(fmaxf(rintf(f[q] * a.inv_out_scale), -127.f), 127.f);
        int8_t* op = static_cast<int8_t*>(a.out) + o;
        if (((a.ldo | a.co_off) & 15) == 0) {
          *reinterpret_cast<i32x4v*>(op) = pk;
        } else {
          for (int q = 0; q < 16; ++q) op[q] = pb[q];
        }
      } else {
        bf16* op = static_cast<bf16*>(a.out) + o;
        bf16x8 o0, o1;
#pragma unroll
        for (int q = 0; q < 8; ++q) { o0[q] = (bf16)f[q]; o1[q] = (bf16)f[q + 8]; }
        if (((a.ldo | a.co_off) & 7) == 0) {
          *reinterpret_cast<bf16x8*>(op) = o0;
          *reinterpret_cast<bf16x8*>(op + 8) = o1;
        } else {
          for (int q = 0; q < 8; ++q) { op[q] = o0[q]; op[q + 8] = o1[q]; }
        }
      }
    } else {  // channel tail (e.g. the 19-class logits)
      for (int q = 0; q < 16 && n + q < a.Cout; ++q) {
        float x = f[q] * a.scale[n + q] + a.bias[n + q];
        if (a.img_bias) x += a.img_bias[(size_t)b * a.Cout + n + q];
        if (a.res) x += (float)a.res[(size_t)m * a.Cout + n + q] * a.res_scale;
        x = apply_act(x, a.act);
        const size_t o = (size_t)m * a.ldo + a.co_off + n + q;
        if (a.out_mode == 0)
          static_cast<int8_t*>(a.out)[o] = (signed char)fminf(fmaxf(rintf(x * a.inv_out_scale), -127.f), 127.f);
        else
          static_cast<bf16*>(a.out)[o] = (bf16)x;
      }
    }
  }
}

template <int MT, int NT>
__global__ __launch_bounds__(256) void conv_i8_kernel(I8Args a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = a.B * a.OH * a.OW;
  const int tiles_m = cdiv_dev(M, 32 * MT), tiles_n = cdiv_dev(a.Cout, 32 * NT);
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  const int pix0 = tm * 32 * MT + wm * 16 * MT;
  const int ch0 = tn * 32 * NT + wn * 16 * NT;
  const int r = lane & 15, kq = lane >> 4;
  int pb[MT], py[MT], px[MT];
  bool pvalid[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = pix0 + i * 16 + r;
    pvalid[i] = m < M;
    const int mm = pvalid[i] ? m : 0;
    pb[i] = mm / (a.OH * a.OW);
    const int rem = mm - pb[i] * a.OH * a.OW;
    py[i] = (rem / a.OW) * a.stride;
    px[i] = (rem % a.OW) * a.stride;
  }
  bool wvalid[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wvalid[j] = (ch0 + j * 16 + r) < a.Cout;
  i32x4v acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = i32x4v{0, 0, 0, 0};
  const i32x4v zero = {0, 0, 0, 0};
  const int taps = a.KH * a.KW;
  const long long wrow = (long long)taps * a.Cin;
  for (int t = 0; t < taps; ++t) {
    const int dy = (t / a.KW - a.KH / 2) * a.dil, dx = (t % a.KW - a.KW / 2) * a.dil;
    long long off[MT];
    bool ok[MT];
    bool any = false;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int iy = py[i] + dy, ix = px[i] + dx;
      ok[i] = pvalid[i] && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
      off[i] = (((long long)pb[i] * a.IH + iy) * a.IW + ix) * a.Cin;
      any |= ok[i];
    }
    if (!__any(any)) continue;
    const int8_t* wt = a.w + (long long)t * a.Cin;
    for (int c0 = 0; c0 < a.Cin; c0 += 64) {
      const int c = c0 + kq * 16;
      const bool cok = c < a.Cin;
      i32x4v bfr[MT], afr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) bfr[i] = (ok[i] && cok) ? ld16(a.in + off[i] + c) : zero;
#pragma unroll
      for (int j = 0; j < NT; ++j)
        afr[j] = (wvalid[j] && cok) ? ld16(wt + (long long)(ch0 + j * 16 + r) * wrow + c) : zero;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr[j], bfr[i], acc[i][j], 0, 0, 0);
    }
  }
  if constexpr (NT == 4) {
    __shared__ __attribute__((aligned(16))) int ep_all[4 * 16 * kEpPitch];
    i8_epilogue_lds<MT>(a, acc, pix0, ch0, ep_all + wid * 16 * kEpPitch, lane);
    return;
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = pix0 + i * 16 + r;
    if (m >= M) continue;
    const int b = pb[i];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = ch0 + j * 16 + kq * 4;
      if (n >= a.Cout) continue;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (n + q >= a.Cout) { v[q] = 0.f; continue; }
        v[q] = (float)acc[i][j][q] * a.scale[n + q] + a.bias[n + q];
        if (a.img_bias) v[q] += a.img_bias[(long long)b * a.Cout + n + q];
        if (a.res) v[q] += (float)a.res[(long long)m * a.Cout + n + q] * a.res_scale;
        v[q] = apply_act(v[q], a.act);
      }
      const long long o = (long long)m * a.ldo + a.co_off + n;
      if (a.out_mode == 0) {
        int8_t* op = static_cast<int8_t*>(a.out) + o;
        char4 pk;
        signed char qv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          qv[q] = (signed char)fminf(fmaxf(rintf(v[q] * a.inv_out_scale), -127.f), 127.f);
        if (n + 3 < a.Cout && ((a.ldo | a.co_off) & 3) == 0) {
          pk = make_char4(qv[0], qv[1], qv[2], qv[3]);
          *reinterpret_cast<char4*>(op) = pk;
        } else {
          for (int q = 0; q < 4; ++q) if (n + q < a.Cout) op[q] = qv[q];
        }
      } else {
        bf16* op = static_cast<bf16*>(a.out) + o;
        for (int q = 0; q < 4; ++q) if (n + q < a.Cout) op[q] = (bf16)v[q];
      }
    }
  }
}

template <int MT, int NT>
void launch_i8(const I8Args& a, hipStream_t s) {
  const int M = a.B * a.OH * a.OW;
  const int grid = cdiv(M, 32 * MT) * cdiv(a.Cout, 32 * NT);
  hipLaunchKernelGGL((conv_i8_kernel<MT, NT>), dim3(grid), dim3(256), 0, s, a);
  check_launch("conv_i8");
}

// ---------------------------------------------------------------------------
// LDS-DMA pipelined int8 variant (the structure of conv_gemm.hip's glds kernel):
// BM x BN tiles, operand rows of 128 K-bytes go global -> LDS with
// buffer_load_dwordx4 ... lds (XOR-swizzled on the source address, padded chunks
// read as zeros through the descriptor's range check), a 2-stage ring with one barrier per 128-deep K step, and
// the 16-byte fragments of v_mfma_i32_16x16x64_i8 read back from LDS. The
// register-fed kernel above loads every fragment from global memory in each wave
// (no reuse across a workgroup's waves); here a 128 x 128 tile's operands are
// fetched once per workgroup.
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// One BM x BN output tile (index bid, row-major over (m-tile, n-tile)); shared by the
// single-conv kernel and the grouped kernel (the int8 ASPP branches in one grid).
// KB: K bytes per stage row. 128 (two MFMA k-steps per stage, 8 rows per glds) or 64 (one
// k-step, 16 rows per glds): half the LDS per stage, so twice the workgroups per CU hide each
// other's global -> LDS round trips -- the short-K convs (layer-4 1x1s, K = 512: four
// 128-deep stages per tile) are latency-bound at two workgroups per CU
template <int MT, int NT, int WM, int WN, int KB = 128>
__device__ __forceinline__ void i8_glds_tile(const I8Args& a, const int bid, char* smem) {
  constexpr int NW = WM * WN, ST = 2;
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN, ROWB = KB;  // KB int8 of K per row
  constexpr int CPR = ROWB / 16, RPG = 1024 / ROWB;  // 16-byte chunks per row, rows per glds
  static_assert(KB == 128 || KB == 64, "KB 128 or 64");
  constexpr int GA = BM / (RPG * NW), GB = BN / (RPG * NW);
  static_assert(GA * RPG * NW == BM && GB * RPG * NW == BN, "tile rows must split over the waves");
  constexpr int SB = (BM + BN) * ROWB;
  int* s_tap = reinterpret_cast<int*>(smem + ST * SB);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int r16 = lane & 15, kq = lane >> 4;
  // GEMM rows: output pixels, or (perm) pixels grouped by tap validity into whole tiles, so
  // the tile tap mask below skips every all-padding tap of the dilated ASPP branches
  const int M = a.perm ? a.Mp : a.B * a.OH * a.OW;
  const int tiles_n = cdiv_dev(a.Cout, BN), tiles_m = cdiv_dev(M, BM);
  const int tn = a.nmajor ? bid / tiles_m : bid % tiles_n;
  const int tm = a.nmajor ? bid - tn * tiles_m : bid / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int taps = a.KH * a.KW;
  const int grow = lane / CPR, lc = (lane % CPR) ^ (grow % CPR);

  // Operand rows come in through buffer_load ... lds on range-checked descriptors (round 5):
  // an out-of-image tap, a channel tail or a row past M gets an offset past the descriptor's
  // end and the hardware writes zeros -- no zero page, no per-row branches or 64-bit
  // address math in the loop. Each A row keeps its 32-bit pixel offset and a mask of the
  // taps that land inside the image; the tap's (dy, dx) offset is one scalar add per step.
  constexpr unsigned kOOB = 0x80000000u;
  const auto rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.in), 0,
                                                     (int)((long long)a.B * a.IH * a.IW * a.Cin), 0x00020000);
  const auto rwt = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.w), 0,
                                                     (int)((long long)a.Cout * taps * a.Cin), 0x00020000);
  unsigned aoff[GA];
  int nrtap[GA];  // taps that fall outside the image (or every tap for a row past M)
  int tapbits = 0;
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int m = m0 + wid * (BM / NW) + i * RPG + grow;
    const int pm = m < M ? (a.perm ? a.perm[m] : m) : -1;
    const int mm = pm >= 0 ? pm : 0;
    const int b = mm / (a.OH * a.OW);
    const int rem = mm - b * a.OH * a.OW;
    const int ay = (rem / a.OW) * a.stride, ax = (rem % a.OW) * a.stride;
    aoff[i] = (unsigned)((((b * a.IH + ay) * a.IW + ax) * a.Cin) + lc * 16);
    const int bits = pm >= 0 ? conv_tap_mask(ay, ax, a.KH, a.KW, a.dil, a.IH, a.IW) : 0;
    nrtap[i] = ~bits;
    tapbits |= bits;
  }
  unsigned boff[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int n = n0 + wid * (BN / NW) + j * RPG + grow;
    boff[j] = n < a.Cout ? (unsigned)(n * taps * a.Cin + lc * 16) : kOOB;
  }
  if (tid == 0) *s_tap = 0;
  __syncthreads();
  if (tapbits) atomicOr(s_tap, tapbits);
  __syncthreads();
  const int tapmask = __builtin_amdgcn_readfirstlane(*s_tap);
  unsigned long long tl = 0;
  int ntap = 0;
  for (int t = 0; t < taps; ++t)
    if ((tapmask >> t) & 1) { tl |= (unsigned long long)t << (4 * ntap); ++ntap; }
  const int cch = cdiv_dev(a.Cin, KB);
  const int total = ntap * cch;
  const int cin_left = a.Cin - lc * 16;  // this lane's 16-byte chunk exists while KB * c < cin_left

  int is_tap = 0, is_c = 0;
  auto issue = [&](int stage) {
    const int t = (int)((tl >> (4 * is_tap)) & 15);
    const int ty = a.KW == 3 ? (t * 11) >> 5 : a.KW == 1 ? t : t / a.KW;
    const int dy = (ty - a.KH / 2) * a.dil, dx = (t - ty * a.KW - a.KW / 2) * a.dil;
    const int cb = is_c * KB;
    // branch-free range handling: bit 31 set = past the descriptor's end (reads zeros)
    const unsigned cbad = (unsigned)(cin_left - cb - 1) & kOOB;
    const unsigned doff = (unsigned)((dy * a.IW + dx) * a.Cin + cb);
    char* sA = smem + stage * SB;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const unsigned vo = (aoff[i] + doff) | cbad | (((unsigned)nrtap[i] << (31 - t)) & kOOB);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_ptr_t)(sA + (wid * (BM / NW) + i * RPG) * ROWB), 16, vo, 0, 0, 0);
    }
    char* sB = sA + BM * ROWB;
    const unsigned wofs = (unsigned)(t * a.Cin + cb);
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const unsigned vo = (boff[j] + wofs) | cbad;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwt, (lds_ptr_t)(sB + (wid * (BN / NW) + j * RPG) * ROWB), 16, vo, 0, 0, 0);
    }
    if (++is_c == cch) { is_c = 0; ++is_tap; }
  };

  i32x4v acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = i32x4v{0, 0, 0, 0};

  if (total > 0) issue(0);
  for (int k = 0; k < total; ++k) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (k + 1 < total) issue((k + 1) % ST);
    const char* sA = smem + (k % ST) * SB;
    const char* sB = sA + BM * ROWB;
    // both K halves' fragments are requested up front: the second half's reads land
    // under the first half's MFMAs
    constexpr int KST = KB / 64;  // MFMA k-steps per stage
    i32x4v bfr[KST][MT], afr[KST][NT];
#pragma unroll
    for (int ks = 0; ks < KST; ++ks) {
      const int kc = ks * 4 + kq;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int r = wm * 16 * MT + i * 16 + r16;
        bfr[ks][i] = *reinterpret_cast<const i32x4v*>(sA + r * ROWB + ((kc ^ (r % CPR)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = wn * 16 * NT + j * 16 + r16;
        afr[ks][j] = *reinterpret_cast<const i32x4v*>(sB + n * ROWB + ((kc ^ (n % CPR)) << 4));
      }
    }
#pragma unroll
    for (int ks = 0; ks < KST; ++ks)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr[ks][j], bfr[ks][i], acc[i][j], 0, 0, 0);
  }

  static_assert(NT == 4, "conv_i8_glds: the LDS epilogue stages 64-channel wave tiles");
  __syncthreads();  // every wave is done reading the last stage: reuse it for the epilogue
  i8_epilogue_lds<MT>(a, acc, m0 + wm * 16 * MT, n0 + wn * 16 * NT,
                      reinterpret_cast<int*>(smem) + wid * 16 * kEpPitch, lane);
}

template <int MT, int NT, int WM, int WN, int KB = 128>
__global__ __launch_bounds__(64 * WM * WN) void conv_i8_glds_kernel(I8Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const int M = a.perm ? a.Mp : a.B * a.OH * a.OW;
  const int tiles = cdiv_dev(M, BM) * cdiv_dev(a.Cout, BN);
  i8_glds_tile<MT, NT, WM, WN, KB>(a, xcd_remap(blockIdx.x, tiles), smem);
}

constexpr int kMaxI8Group = 4;
struct I8GroupArgs {
  I8Args g[kMaxI8Group];
  const int* order;
};

template <int MT, int NT, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void conv_i8_glds_group_kernel(I8GroupArgs ga) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int e = __builtin_amdgcn_readfirstlane(ga.order[blockIdx.x]);
  const int t = e & 0xffffff;
  switch (e >> 24) {  // constant indices: each arm reads its I8Args straight from kernarg
    case 0: i8_glds_tile<MT, NT, WM, WN>(ga.g[0], t, smem); break;
    case 1: i8_glds_tile<MT, NT, WM, WN>(ga.g[1], t, smem); break;
    case 2: i8_glds_tile<MT, NT, WM, WN>(ga.g[2], t, smem); break;
    default: i8_glds_tile<MT, NT, WM, WN>(ga.g[3], t, smem); break;
  }
}

template <int MT, int NT, int WM, int WN>
void launch_i8_glds_group(const I8GroupArgs& ga, int nblocks, hipStream_t s) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const size_t lds = 2 * (size_t)(BM + BN) * 128 + 16;
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_i8_glds_group_kernel<MT, NT, WM, WN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "conv_i8_glds_group attr");
    attr = true;
  }
  hipLaunchKernelGGL((conv_i8_glds_group_kernel<MT, NT, WM, WN>), dim3(nblocks), dim3(64 * WM * WN), lds, s, ga);
  check_launch("conv_i8_glds_group");
}

template <int MT, int NT, int WM, int WN, int KB = 128>
void launch_i8_glds(const I8Args& a, hipStream_t s) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const int M = a.perm ? a.Mp : a.B * a.OH * a.OW;
  const int grid = cdiv(M, BM) * cdiv(a.Cout, BN);
  // the epilogue stages every wave's 16 x 64 int32 tile in the ring's bytes
  static_assert(2 * (BM + BN) * KB >= WM * WN * 16 * kEpPitch * 4, "epilogue staging exceeds the ring");
  const size_t lds = 2 * (size_t)(BM + BN) * KB + 16;
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_i8_glds_kernel<MT, NT, WM, WN, KB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "conv_i8_glds attr");
    attr = true;
  }
  hipLaunchKernelGGL((conv_i8_glds_kernel<MT, NT, WM, WN, KB>), dim3(grid), dim3(64 * WM * WN), lds, s, a);
  check_launch("conv_i8_glds");
}

// ---- int8 helpers: max pool and global average pool on int8 NHWC
__global__ void maxpool_i8_kernel(const int8_t* __restrict__ in, int8_t* __restrict__ out, int B,
                                  int IH, int IW, int C, int OH, int OW) {
  const int CG = C >> 4;
  const long long total = (long long)B * OH * OW * CG;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int cg = (int)(t % CG);
  long long pix = t / CG;
  const int ox = (int)(pix % OW);
  pix /= OW;
  const int oy = (int)(pix % OH);
  const int b = (int)(pix / OH);
  signed char m[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) m[q] = -128;
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * 2 + ky - 1;
    if (iy < 0 || iy >= IH) continue;
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ox * 2 + kx - 1;
      if (ix < 0 || ix >= IW) continue;
      const int4 v = *reinterpret_cast<const int4*>(in + (((long long)b * IH + iy) * IW + ix) * C + cg * 16);
      const signed char* pv = reinterpret_cast<const signed char*>(&v);
#pragma unroll
      for (int q = 0; q < 16; ++q) m[q] = pv[q] > m[q] ? pv[q] : m[q];
    }
  }
  *reinterpret_cast<int4*>(out + t * 16) = *reinterpret_cast<int4*>(m);
}

__global__ __launch_bounds__(256) void gap_i8_kernel(const int8_t* __restrict__ in, float* __restrict__ part,
                                                     int HW, int C, int slices) {
  const int b = blockIdx.x, sl = blockIdx.y;
  const int c = blockIdx.z * 256 + threadIdx.x;
  if (c >= C) return;
  const int p0 = (int)((long long)HW * sl / slices), p1 = (int)((long long)HW * (sl + 1) / slices);
  int s = 0;
  for (int p = p0; p < p1; ++p) s += in[((long long)b * HW + p) * C + c];
  part[((long long)b * slices + sl) * C + c] = (float)s;
}

// Vectorised form (C % 16 == 0): a thread sums 16 channels of every PH-th pixel of the
// slice from 16-byte loads (four in flight), the PH pixel phases of a workgroup meet in LDS.
// The byte-per-thread kernel above issued one dependent 1-byte load per pixel: 67 us for the
// config-4 ASPP pool (B = 8, 65 x 65 x 2048 int8, 69 MB) against ~14 us of HBM time.
template <int CGN, int PH>
__global__ __launch_bounds__(256) void gap_i8_vec_kernel(const int8_t* __restrict__ in, float* __restrict__ part,
                                                         int HW, int C, int slices) {
  static_assert(CGN * PH == 256, "one thread per (channel group, pixel phase)");
  __shared__ __attribute__((aligned(16))) int red[PH * CGN * 16];
  const int b = blockIdx.x, sl = blockIdx.y;
  const int cg = threadIdx.x % CGN, ph = threadIdx.x / CGN;
  const int cb = blockIdx.z * CGN * 16;
  const int c0 = cb + cg * 16;
  const int p0 = (int)((long long)HW * sl / slices), p1 = (int)((long long)HW * (sl + 1) / slices);
  int acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0;
  auto add = [&](const i32x4v v) {
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[w * 4 + k] += (v[w] << (24 - 8 * k)) >> 24;
  };
  if (c0 < C) {
    const int8_t* src = in + (long long)b * HW * C + c0;
    int p = p0 + ph;
    for (; p + 3 * PH < p1; p += 4 * PH) {
      const i32x4v v0 = ld16(src + (long long)p * C), v1 = ld16(src + (long long)(p + PH) * C);
      const i32x4v v2 = ld16(src + (long long)(p + 2 * PH) * C), v3 = ld16(src + (long long)(p + 3 * PH) * C);
      add(v0); add(v1); add(v2); add(v3);
    }
    for (; p < p1; p += PH) add(ld16(src + (long long)p * C));
  }
#pragma unroll
  for (int q = 0; q < 16; q += 4)
    *reinterpret_cast<i32x4v*>(red + (ph * CGN + cg) * 16 + q) = i32x4v{acc[q], acc[q + 1], acc[q + 2], acc[q + 3]};
  __syncthreads();
  for (int i = threadIdx.x; i < CGN * 16; i += 256) {
    if (cb + i >= C) break;
    int t = 0;
#pragma unroll
    for (int k = 0; k < PH; ++k) t += red[k * CGN * 16 + i];
    part[((long long)b * slices + sl) * C + cb + i] = (float)t;
  }
}

__global__ void gap_i8_reduce(const float* __restrict__ part, float* __restrict__ out, int B, int C,
                              int slices, float scale) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i % C;
  float s = 0.f;
  for (int k = 0; k < slices; ++k) s += part[((long long)b * slices + k) * C + c];
  out[i] = s * scale;
}

}  // namespace

// ---------------------------------------------------------------------------
// Streaming 1x1 variant (any stride; 3x3 form below) for the memory-bound bottleneck convs (ResNet-50
// layers 1-3 at 1025^2: K = 64..256, 2-27 MAC per byte moved). The register-fed kernel
// above runs one short-lived 32x32..32x64 tile per wave with the weights reloaded from
// L2 by every wave and a 4-byte-per-lane epilogue (r4_config4_roofline.txt: L1's 1x1 convs
// at 12-31 % of HBM bandwidth). Here a workgroup owns one block of NB = 16 NS output
// channels for its whole life: the block's weight fragments are loaded into VGPRs once,
// then the workgroup walks pixel tiles of 64 (one 16-pixel subtile per wave), prefetching
// the next tile's input fragments while the MFMAs of the current one run, and stages the
// int32 accumulators through LDS so the epilogue reads 16 consecutive channels of one
// pixel per lane (16-byte residual loads and stores). Exact int32 accumulation; the int8
// epilogue folds the requantisation into the affine terms (see below: within one rounding
// step of the other variants), the bf16 one is theirs.
template <int CF, int NS, int PD, int KT, bool WL = false>
__global__ __launch_bounds__(256) void conv_i8_1x1_kernel(I8Args a, int nblk) {
  // WL: the weight fragments live in LDS (NS * KF KiB, one conflict-free ds_read_b128 per
  // MFMA) instead of VGPRs -- fewer registers, more resident waves for the 3x3 form
  // KT = 1 (1x1, stride 1) or 9 (3x3, any stride / dilation: the taps are extra K fragments
  // read from the shifted pixels, zero outside the image)
  constexpr int KF = KT * CF;           // K fragments of 64 per output pixel
  constexpr int NB = 16 * NS;           // output channels per workgroup
  constexpr int EPP = NB + 4;           // staged row pitch (ints): 16 distinct bank groups
  __shared__ __attribute__((aligned(16))) int ep_all[4 * 16 * EPP];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
  const int M = a.B * a.OH * a.OW;
  const int nb = blockIdx.x % nblk;     // this workgroup's channel block
  const int tstep = gridDim.x / nblk;   // (the grid is a multiple of nblk)
  const int ch0 = nb * NB;
  // weights: A fragments (rows = out channels, 16 K bytes per lane), resident
  constexpr int NWF = WL ? 1 : NS, KWF = WL ? 1 : KF;
  i32x4v wf[NWF][KWF];
  __shared__ __attribute__((aligned(16))) i32x4v s_w[WL ? NS * KF * 64 : 1];
  if constexpr (WL) {
    for (int i = threadIdx.x; i < NS * KF * 64; i += 256) {
      const int l = i & 63, jf = i >> 6, j = jf / KF, f = jf - j * KF;
      s_w[i] = ld16(a.w + (size_t)(ch0 + j * 16 + (l & 15)) * KT * a.Cin + (f / CF) * a.Cin + (f % CF) * 64 +
                    (l >> 4) * 16);
    }
  } else {
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int f = 0; f < KF; ++f)  // [Cout][tap][Cin]: fragment f = tap * CF + (f % CF)
        wf[j][f] = ld16(a.w + (size_t)(ch0 + j * 16 + r) * KT * a.Cin + (f / CF) * a.Cin + (f % CF) * 64 + kq * 16);
  }
  int* ep = ep_all + wid * 16 * EPP;
  // the block's requantisation constants in LDS (int8 out: folded as in i8_requant16)
  __shared__ __attribute__((aligned(16))) float s_sc[NB], s_bi[NB];
  const float ios = a.inv_out_scale;
  const float rs = a.res ? a.res_scale * ios : 0.f;
  for (int i = threadIdx.x; i < NB; i += 256) {
    s_sc[i] = a.scale[ch0 + i] * ios;
    s_bi[i] = fmaf(a.bias[ch0 + i], ios, 128.f - 128.f * rs);
  }
  __syncthreads();
  const float lo = a.act == ACT_NONE ? 1.f : 128.f;
  const float hi = a.act == ACT_RELU6 ? fminf(255.f, 128.f + 6.f * ios) : 255.f;
  const int ntile = (M + 63) / 64;
  int t = blockIdx.x / nblk;
  i32x4v xf[PD][KF];  // PD tiles of input fragments in flight
  auto load_x = [&](int tile, i32x4v (&dst)[KF]) {
    const int m = min(tile * 64 + wid * 16 + r, M - 1);  // clamped: tail pixels are not stored
    if constexpr (KT == 1) {
      size_t pix = (size_t)m;
      if (a.stride != 1) {  // strided 1x1 (the projection shortcuts): the sampled input pixel
        const int b = m / (a.OH * a.OW), rem = m - b * a.OH * a.OW;
        const int oy = rem / a.OW, ox = rem - oy * a.OW;
        pix = ((size_t)b * a.IH + oy * a.stride) * a.IW + ox * a.stride;
      }
#pragma unroll
      for (int f = 0; f < CF; ++f) dst[f] = ld16(a.in + pix * a.Cin + f * 64 + kq * 16);
    } else {
      const int b = m / (a.OH * a.OW), rem = m - b * a.OH * a.OW;
      const int oy = rem / a.OW, ox = rem - oy * a.OW;
#pragma unroll
      for (int tp = 0; tp < KT; ++tp) {
        const int iy = oy * a.stride + (tp / 3 - 1) * a.dil, ix = ox * a.stride + (tp % 3 - 1) * a.dil;
        const bool ok = iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
        const int8_t* src = a.in + (((size_t)b * a.IH + (ok ? iy : 0)) * a.IW + (ok ? ix : 0)) * a.Cin + kq * 16;
#pragma unroll
        for (int f = 0; f < CF; ++f) dst[tp * CF + f] = ok ? ld16(src + f * 64) : i32x4v{0, 0, 0, 0};
      }
    }
  };
  const int px = lane >> 2, cq = lane & 3;  // epilogue: 16 pixels x 4 lanes of 16 channels
  // one tile: MFMAs on xb, staged transpose, epilogue
  constexpr int NG = (NS + 3) / 4;  // 16-channel groups per epilogue lane
  auto tile_work = [&](int tile, const i32x4v (&xb)[KF]) {
    // this lane's residual bytes for the epilogue, in flight under the MFMAs
    const int me = tile * 64 + wid * 16 + px;
    i32x4v rq[NG];
    if (a.res && a.out_mode == 0) {
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        const int g = cq + 4 * i;
        rq[i] = (g < NS && me < M) ? *reinterpret_cast<const i32x4v*>(a.res + (size_t)me * a.Cout + ch0 + g * 16)
                                   : i32x4v{0, 0, 0, 0};
      }
    }
    i32x4v acc[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      acc[j] = i32x4v{0, 0, 0, 0};
#pragma unroll
      for (int f = 0; f < KF; ++f) {
        const i32x4v wa = WL ? s_w[(j * KF + f) * 64 + lane] : wf[WL ? 0 : j][WL ? 0 : f];
        acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wa, xb[f], acc[j], 0, 0, 0);
      }
    }
    // stage [16 px][NB ch]: lane (r = pixel, kq) holds channels j*16 + kq*4 .. +3
#pragma unroll
    for (int j = 0; j < NS; ++j) *reinterpret_cast<i32x4v*>(ep + r * EPP + j * 16 + kq * 4) = acc[j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int m = tile * 64 + wid * 16 + px;
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {  // this lane's 16-channel groups of pixel px
      const int g = cq + 4 * gi;
      if (g >= NS) break;
      i32x4v v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = *reinterpret_cast<const i32x4v*>(ep + px * EPP + g * 16 + c * 4);
      if (m >= M) continue;
      const int n = ch0 + g * 16;
      const size_t o = (size_t)m * a.ldo + a.co_off + n;
      if (a.out_mode == 0 && !a.img_bias) {
        // int8 out: the folded requantisation (i8_requant16) with the block's constants from
        // LDS and the residual prefetched above
        i32x4v pk;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 sc = *reinterpret_cast<const float4*>(s_sc + g * 16 + c * 4);
          const float4 bi = *reinterpret_cast<const float4*>(s_bi + g * 16 + c * 4);
          const float s4[4] = {sc.x, sc.y, sc.z, sc.w}, b4[4] = {bi.x, bi.y, bi.z, bi.w};
          const unsigned ur = a.res ? ((unsigned)rq[gi][c] ^ 0x80808080u) : 0u;
          unsigned w = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float z = fmaf((float)v[c][q], s4[q], b4[q]);
            if (a.res) z = fmaf((float)((ur >> (8 * q)) & 0xffu), rs, z);
            z = __builtin_amdgcn_fmed3f(z, lo, hi);
            w = __builtin_amdgcn_cvt_pk_u8_f32(z, q, w);
          }
          pk[c] = (int)(w ^ 0x80808080u);
        }
        *reinterpret_cast<i32x4v*>(static_cast<int8_t*>(a.out) + o) = pk;
        continue;
      }
      if (a.out_mode == 0) {  // int8 out with a per-image bias
        *reinterpret_cast<i32x4v*>(static_cast<int8_t*>(a.out) + o) = i8_requant16(a, v, m, n);
        continue;
      }
      float f[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 sc = *reinterpret_cast<const float4*>(a.scale + n + c * 4);
        const float4 bi = *reinterpret_cast<const float4*>(a.bias + n + c * 4);
        f[c * 4 + 0] = (float)v[c][0] * sc.x + bi.x; f[c * 4 + 1] = (float)v[c][1] * sc.y + bi.y;
        f[c * 4 + 2] = (float)v[c][2] * sc.z + bi.z; f[c * 4 + 3] = (float)v[c][3] * sc.w + bi.w;
        if (a.img_bias) {
          const int b = m / (a.OH * a.OW);
          const float4 ib = *reinterpret_cast<const float4*>(a.img_bias + (size_t)b * a.Cout + n + c * 4);
          f[c * 4 + 0] += ib.x; f[c * 4 + 1] += ib.y; f[c * 4 + 2] += ib.z; f[c * 4 + 3] += ib.w;
        }
      }
      if (a.res) {
        const i32x4v rv = *reinterpret_cast<const i32x4v*>(a.res + (size_t)m * a.Cout + n);
        const signed char* rb = reinterpret_cast<const signed char*>(&rv);
#pragma unroll
        for (int q = 0; q < 16; ++q) f[q] += (float)rb[q] * a.res_scale;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) f[q] = apply_act(f[q], a.act);
      bf16* op = static_cast<bf16*>(a.out) + o;
      bf16x8 o0, o1;
#pragma unroll
      for (int q = 0; q < 8; ++q) { o0[q] = (bf16)f[q]; o1[q] = (bf16)f[q + 8]; }
      *reinterpret_cast<bf16x8*>(op) = o0;
      *reinterpret_cast<bf16x8*>(op + 8) = o1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the next tile rewrites ep
  };
  // PD tiles per iteration, so the prefetch buffers stay statically indexed
#pragma unroll
  for (int i = 0; i < PD - 1; ++i)
    if (t + i * tstep < ntile) load_x(t + i * tstep, xf[i]);
#pragma unroll 1
  for (; t < ntile; t += PD * tstep) {
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int tt = t + i * tstep;
      if (tt >= ntile) break;
      const int tp = tt + (PD - 1) * tstep;
      if (tp < ntile) load_x(tp, xf[(i + PD - 1) % PD]);
      tile_work(tt, xf[i]);
    }
  }
}

template <int CF, int NS, int KT = 1, bool WL = false>
void launch_i8_1x1(const I8Args& a, hipStream_t s) {
  const int M = a.B * a.OH * a.OW;
  const int nblk = a.Cout / (16 * NS);
  const int ntile = cdiv(M, 64);
  // ~4 resident workgroups per CU, each channel block's tiles spread over the same count
  const int per = std::max(1, std::min(ntile, 1024 / nblk));
  // prefetch depth: input tiles in flight per wave (CF * 4 VGPRs each)
  constexpr int KF = KT * CF;
  // (the LDS-weight 3x3 form keeps no tile in flight: its 9 * CF input fragments per tile
  // would double the registers; occupancy hides the latency instead)
  constexpr int PD = KT > 1 ? (WL ? 1 : 2) : (KF * NS > 32 ? 2 : (KF <= 2 ? 4 : (KF <= 4 ? 3 : 2)));
  hipLaunchKernelGGL((conv_i8_1x1_kernel<CF, NS, PD, KT, WL>), dim3(per * nblk), dim3(256), 0, s, a, nblk);
  check_launch("conv_i8_1x1");
}

// (CF, NS): K fragments of 64 per pixel, 16-channel subtiles per workgroup; NS * CF <= 16
// keeps the weight fragments at <= 64 VGPRs. First match wins (widest channel block).
constexpr int kI8x1Inst[][2] = {{1, 16}, {1, 8}, {1, 4}, {2, 16}, {2, 8}, {2, 4}, {4, 16}, {4, 8}, {4, 4}, {4, 2},
                                 {8, 8}, {8, 4}, {8, 2}, {8, 1}, {16, 4}, {16, 2}, {16, 1}};

// 3x3 (KT = 9), weights in VGPRs: 9 * CF * NS <= 36 fragments (144 VGPRs), Cin <= 128;
// weights in LDS (WL): NS * 9 * CF KiB <= 72
constexpr int kI8x3Inst[][2] = {{1, 4}, {1, 2}, {2, 2}, {2, 1}};
constexpr int kI8x3InstL[][2] = {{1, 8}, {1, 4}, {2, 4}, {2, 2}, {4, 2}, {4, 1}};

void launch_i8_3x3_any(const I8Args& a, hipStream_t s, int which) {
  const int CF = a.Cin / 64, nsub = a.Cout / 16;
  // variants 10 / 11: the LDS-weight form; either form falls back to the other when it has
  // no instantiation for this (Cin, Cout)
  auto collect = [&](bool l, int (&fit)[8]) {
    int n = 0;
    if (l) {
      for (const auto& cn : kI8x3InstL)
        if (cn[0] == CF && nsub % cn[1] == 0 && n < 8) fit[n++] = cn[1];
    } else {
      for (const auto& cn : kI8x3Inst)
        if (cn[0] == CF && nsub % cn[1] == 0 && n < 8) fit[n++] = cn[1];
    }
    return n;
  };
  bool wl = which >= 2;
  int fit[8];
  int nf = collect(wl, fit);
  if (nf == 0) {
    wl = !wl;
    nf = collect(wl, fit);
  }
  if (nf == 0) throw std::invalid_argument("conv_i8: no 3x3 streaming instantiation for this Cin / Cout");
  const int ns = fit[std::min(which & 1, nf - 1)];
#define I8_3X3(CF_, NS_)                                    \
  if (!wl && CF == CF_ && ns == NS_) { launch_i8_1x1<CF_, NS_, 9>(a, s); return; }
#define I8_3X3L(CF_, NS_)                                   \
  if (wl && CF == CF_ && ns == NS_) { launch_i8_1x1<CF_, NS_, 9, true>(a, s); return; }
  I8_3X3(1, 4) I8_3X3(1, 2) I8_3X3(2, 2) I8_3X3(2, 1)
  I8_3X3L(1, 8) I8_3X3L(1, 4) I8_3X3L(2, 4) I8_3X3L(2, 2) I8_3X3L(4, 2) I8_3X3L(4, 1)
#undef I8_3X3
#undef I8_3X3L
  throw std::invalid_argument("conv_i8: no 3x3 streaming instantiation for this Cin / Cout");
}

void launch_i8_1x1_any(const I8Args& a, hipStream_t s, int which) {
  const int CF = a.Cin / 64, nsub = a.Cout / 16;
  // the fitting instantiations of this CF, widest channel block first; `which` (variants
  // 5, 6, 10, 11 -> 0..3) picks one: narrower blocks hold fewer weight / accumulator VGPRs
  // and read the input once more per extra block (from L2)
  int fit[8], nf = 0;
  for (const auto& cn : kI8x1Inst)
    if (cn[0] == CF && nsub % cn[1] == 0 && nf < 8) fit[nf++] = cn[1];
  if (nf == 0) throw std::invalid_argument("conv_i8: no 1x1 streaming instantiation for this Cin / Cout");
  const int ns = fit[std::min(which, nf - 1)];
#define I8_1X1(CF_, NS_)                                    \
  if (CF == CF_ && ns == NS_) { launch_i8_1x1<CF_, NS_>(a, s); return; }
  I8_1X1(1, 16) I8_1X1(1, 8) I8_1X1(1, 4) I8_1X1(2, 16) I8_1X1(2, 8) I8_1X1(2, 4) I8_1X1(4, 16)
  I8_1X1(4, 8) I8_1X1(4, 4) I8_1X1(4, 2) I8_1X1(8, 8) I8_1X1(8, 4) I8_1X1(8, 2) I8_1X1(8, 1)
  I8_1X1(16, 4) I8_1X1(16, 2) I8_1X1(16, 1)
#undef I8_1X1
  throw std::invalid_argument("conv_i8: no 1x1 streaming instantiation for this Cin / Cout");
}

bool conv_i8_1x1_ok(const ConvI8Params& p) {
  const int CF = p.Cin / 64, nsub = p.Cout / 16;
  const bool k3 = p.KH == 3 && p.KW == 3;
  bool inst = false;
  if (k3) {
    for (const auto& cn : kI8x3Inst)
      if (CF == cn[0] && nsub % cn[1] == 0) inst = true;
    for (const auto& cn : kI8x3InstL)
      if (CF == cn[0] && nsub % cn[1] == 0) inst = true;
  } else {
    for (const auto& cn : kI8x1Inst)
      if (CF == cn[0] && nsub % cn[1] == 0) inst = true;
  }
  const int vec = p.out_mode == 0 ? 16 : 8;  // 16-byte stores
  const bool geom = k3 || (p.KH == 1 && p.KW == 1 && p.OH == (p.IH - 1) / p.stride + 1 &&
                           p.OW == (p.IW - 1) / p.stride + 1);
  return geom && p.Cin % 64 == 0 && p.Cout % 16 == 0 && (p.ldo % vec) == 0 && (p.co_off % vec) == 0 && inst;
}

static I8Args i8_args(const ConvI8Params& p) {
  if (p.Cin % 16) throw std::invalid_argument("conv_i8: Cin must be a multiple of 16");
  if (p.ldo < p.co_off + p.Cout) throw std::invalid_argument("conv_i8: bad ldo/co_off");
  if (p.perm && p.Mp <= 0) throw std::invalid_argument("conv_i8: perm needs Mp > 0");
  return I8Args{p.in, p.w, p.scale, p.bias, p.img_bias, p.res, p.res_scale, p.out, p.inv_out_scale,
                p.out_mode, p.B, p.IH, p.IW, p.Cin, p.OH, p.OW, p.Cout, p.KH, p.KW, p.stride, p.dil,
                p.ldo, p.co_off, p.act, p.perm, p.perm ? p.Mp : 0, 0};
}

// the LDS-DMA kernels address both operands through 32-bit buffer offsets below 2^31
static bool i8_glds_ok(const ConvI8Params& p) {
  return p.KH * p.KW <= 16 && (long long)p.B * p.IH * p.IW * p.Cin < (1LL << 31) &&
         (long long)p.Cout * p.KH * p.KW * p.Cin < (1LL << 31);
}

void conv_i8_grouped(const ConvI8Params* ps, int n, const int* order, int nblocks, int variant,
                     hipStream_t s) {
  if (n < 1 || n > kMaxI8Group) throw std::invalid_argument("conv_i8_grouped: 1..4 convs");
  if (!order || nblocks <= 0) throw std::invalid_argument("conv_i8_grouped: empty order table");
  I8GroupArgs ga{};
  for (int i = 0; i < n; ++i) {
    if (!i8_glds_ok(ps[i])) throw std::invalid_argument("conv_i8_grouped: conv does not fit the LDS-DMA kernel");
    ga.g[i] = i8_args(ps[i]);
  }
  for (int i = n; i < kMaxI8Group; ++i) ga.g[i] = ga.g[0];
  ga.order = order;
  switch (variant) {
    case 2: launch_i8_glds_group<4, 4, 2, 2>(ga, nblocks, s); return;
    case 3: launch_i8_glds_group<4, 4, 2, 4>(ga, nblocks, s); return;
    case 4: launch_i8_glds_group<4, 4, 4, 2>(ga, nblocks, s); return;
    case 7: launch_i8_glds_group<5, 4, 2, 2>(ga, nblocks, s); return;
    case 8: launch_i8_glds_group<3, 4, 2, 2>(ga, nblocks, s); return;
    default: throw std::invalid_argument("conv_i8_grouped: variant must be 2, 3, 4, 7 or 8");
  }
}

void conv_i8(const ConvI8Params& p, hipStream_t s) {
  I8Args a = i8_args(p);
  const long long M = (long long)p.B * p.OH * p.OW;
  // variant: 0 auto, 1 register-fed, 2 LDS-DMA 128 x 128 (4 waves), 3 LDS-DMA
  // 128 x 256 (8 waves), 4 LDS-DMA 256 x 128 (8 waves), 7 / 8 LDS-DMA 160 x 128 / 96 x 128
  // (4 waves: tile counts that fill the 2-per-CU slots without a near-empty last round), 12 / 13
  // = 7 / 2 with n-tile-major block order, 5 / 6 / 10 / 11 streaming 1x1 (stride 1,
  // Cin % 64 == 0, Cout % 16 == 0, 16-byte aligned output; the widest fitting channel block,
  // then the next narrower ones)
  const bool glds_ok = i8_glds_ok(p);
  int v = p.variant;
  if (v == 12 || v == 13) {  // n-tile-major forms of 7 / 2 (weight-heavy convs: the ASPP 3x3s)
    a.nmajor = 1;
    v = v == 12 ? 7 : 2;
  }
  if (v == 0) v = (glds_ok && p.Cout >= 64 && M >= 8192) ? (p.Cout >= 256 ? 3 : 2) : 1;
  const bool glds_v = (v >= 2 && v <= 4) || v == 7 || v == 8 || (v >= 18 && v <= 20);
  if (glds_v && !glds_ok) throw std::invalid_argument("conv_i8: LDS-DMA variants need <= 16 taps and < 2 GiB operands");
  if (p.perm && !glds_v) throw std::invalid_argument("conv_i8: a row permutation needs an LDS-DMA variant");
  if (v == 5 || v == 6 || v == 10 || v == 11) {
    if (!conv_i8_1x1_ok(p)) throw std::invalid_argument("conv_i8: streaming 1x1 variant does not fit this conv");
    const int which = v == 5 ? 0 : v == 6 ? 1 : v == 10 ? 2 : 3;
    if (p.KH == 3) launch_i8_3x3_any(a, s, which);
    else launch_i8_1x1_any(a, s, which);
    return;
  }
  switch (v) {
    case 2: launch_i8_glds<4, 4, 2, 2>(a, s); return;
    case 3: launch_i8_glds<4, 4, 2, 4>(a, s); return;
    case 4: launch_i8_glds<4, 4, 4, 2>(a, s); return;
    case 7: launch_i8_glds<5, 4, 2, 2>(a, s); return;
    case 8: launch_i8_glds<3, 4, 2, 2>(a, s); return;
    // 64-byte K rows (one k-step per stage, half the LDS): 128 x 128 / 128 x 256 / 256 x 128
    case 18: launch_i8_glds<4, 4, 2, 2, 64>(a, s); return;
    case 19: launch_i8_glds<4, 4, 2, 4, 64>(a, s); return;
    case 20: launch_i8_glds<4, 4, 4, 2, 64>(a, s); return;
    default: break;
  }
  if (p.Cout <= 32) launch_i8<4, 1>(a, s);
  else if (p.Cout <= 64 || M < 8192) launch_i8<2, 2>(a, s);
  else launch_i8<2, 4>(a, s);
}

void maxpool3x3s2_i8(const int8_t* in, int8_t* out, int B, int IH, int IW, int C, int OH, int OW,
                     hipStream_t s) {
  if (C % 16) throw std::invalid_argument("maxpool_i8: C % 16");
  const long long total = (long long)B * OH * OW * (C / 16);
  hipLaunchKernelGGL(maxpool_i8_kernel, dim3(cdiv(total, 256)), dim3(256), 0, s, in, out, B, IH, IW,
                     C, OH, OW);
  check_launch("maxpool_i8");
}

void global_avgpool_i8(const int8_t* in, float* out, float* ws, int B, int HW, int C, float scale,
                       hipStream_t s) {
  const int slices = 16;  // the caller's ws holds B * 16 * C partial sums
  if (C % 16 == 0)
    hipLaunchKernelGGL((gap_i8_vec_kernel<32, 8>), dim3(B, slices, cdiv(C, 512)), dim3(256), 0, s, in, ws, HW,
                       C, slices);
  else
    hipLaunchKernelGGL(gap_i8_kernel, dim3(B, slices, cdiv(C, 256)), dim3(256), 0, s, in, ws, HW, C,
                       slices);
  hipLaunchKernelGGL(gap_i8_reduce, dim3(cdiv((long long)B * C, 256)), dim3(256), 0, s, ws, out, B,
                     C, slices, scale / (float)HW);
  check_launch("gap_i8");
}

}  // namespace ssa
