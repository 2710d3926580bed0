// Implicit-GEMM convolution on MFMA (gfx950), NHWC bf16 in/out, fp32 accumulate.
//
//   out[b, oy, ox, co_off + n] = act( sum_{ky,kx,c} W[n][ky][kx][c] * in[b, iy, ix, c]
//                                     + bias[n] + img_bias[b][n] + res[b, oy, ox, n] )
//   iy = oy*stride + (ky - KH/2)*dil, ix = ox*stride + (kx - KW/2)*dil, zero outside.
//
// Covers every dense conv of the models: MobileNetV2 1x1 expand/project (fused
// residual), ASPP 1x1 / 3x3 atrous branches (written straight into their channel
// slice of the concat buffer: concat-free), the ASPP projection (the image-pool
// branch enters as a per-image bias), the logits layer, and the ResNet-50
// bottleneck 1x1/3x3 (strided) convs.
//
// Mapping: the MFMA's A operand is the weight tile (rows = output channels) and
// the B operand is the pixel tile, so each lane's accumulator holds 4 consecutive
// output channels of one pixel (v_mfma_f32_16x16x32_bf16 C/D layout: row =
// (lane>>4)*4 + r, col = lane&15) and the epilogue stores 8 contiguous bytes.
// Both operands are 16-byte vector loads straight to VGPRs in the MFMA fragment
// layout (lane l: 8 consecutive K elements at k = 8*(l>>4), row/col l&15); taps
// that fall entirely outside the image for all of a wave's pixels are skipped
// (wave-uniform), which removes most of the zero work of the rate-12/18 ASPP
// branches on a 33x33 map.
//
// Block: 4 waves in a 2x2 arrangement; wave tile = (16*MT pixels) x (16*NT chans).
#include "common.h"
#include "kernels.h"

namespace ssa {

struct ConvArgs {
  const bf16* in; const bf16* w; const float* bias; const float* img_bias;
  const bf16* res; bf16* out;
  int B, IH, IW, Cin, OH, OW, Cout;
  int KH, KW, stride, dil;
  int ldo, co_off, ldr, act;
  const int* perm;  // LDS-DMA kernel only: GEMM row -> output pixel (-1: padding), or null
  int Mp;           // rows of the permuted GEMM (perm != null)
};

constexpr int kMaxConvGroup = 4;
struct ConvGroupArgs {
  ConvArgs g[kMaxConvGroup];
  const int* order;  // [nblocks] (group << 24) | (K slice << 20) | tile
  int ks;            // K slices per tile (split-K for small batches); 1 = no split
  float* part;       // ks > 1: fp32 partials [ks][B * OH * OW][ldo] (no bias / act), else null
  int* cnt;          // ks > 1, in-launch combine: per-tile tickets [group][cnt_stride], else null
  int cnt_stride;
};

template <int MT, int NT>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = a.B * a.OH * a.OW;
  const int tiles_m = cdiv_dev(M, 32 * MT);
  const int tiles_n = cdiv_dev(a.Cout, 32 * NT);
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  const int pix0 = tm * 32 * MT + wm * 16 * MT;
  const int ch0 = tn * 32 * NT + wn * 16 * NT;
  const int r = lane & 15, kq = lane >> 4;  // fragment row/col and K quarter

  // per-subtile pixel coordinates for this lane's B-fragment column
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
  // weight rows for this lane's A-fragment
  bool wvalid[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wvalid[j] = (ch0 + j * 16 + r) < a.Cout;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int taps = a.KH * a.KW;
  const long long wrow = (long long)taps * a.Cin;  // weight elements per out channel
  for (int t = 0; t < taps; ++t) {
    const int dy = (t / a.KW - a.KH / 2) * a.dil;
    const int dx = (t % a.KW - a.KW / 2) * a.dil;
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
    if (!__any(any)) continue;  // wave-uniform skip of an all-padding tap
    const bf16* wt = a.w + (long long)t * a.Cin;
    for (int c0 = 0; c0 < a.Cin; c0 += 32) {
      const int c = c0 + kq * 8;
      const bool cok = c < a.Cin;
      bf16x8 bfr[MT], afr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        bfr[i] = (ok[i] && cok) ? ld8(a.in + off[i] + c) : zero8();
#pragma unroll
      for (int j = 0; j < NT; ++j)
        afr[j] = (wvalid[j] && cok) ? ld8(wt + (long long)(ch0 + j * 16 + r) * wrow + c) : zero8();
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[j], bfr[i], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: lane holds out channels ch0 + j*16 + kq*4 + {0..3} of pixel pix0 + i*16 + r
  // (8-byte row pieces; staging the tile through LDS for 16-byte stores measured
  // 1.5x slower on the MobileNetV2 expansions: the extra barrier + LDS round trip
  // costs more than the partial-line writes, which L2 merges)
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = pix0 + i * 16 + r;
    if (m >= M) continue;
    const int b = pb[i];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = ch0 + j * 16 + kq * 4;
      if (n >= a.Cout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      const bool full = n + 3 < a.Cout;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (n + q < a.Cout) {
          v[q] += a.bias[n + q];
          if (a.img_bias) v[q] += a.img_bias[(long long)b * a.Cout + n + q];
        }
      }
      if (a.res) {
        const bf16* rp = a.res + (long long)m * a.ldr + n;
        if (full && (a.ldr & 3) == 0) {
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(rp);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += (float)rv[q];
        } else {
          for (int q = 0; q < 4; ++q) if (n + q < a.Cout) v[q] += (float)rp[q];
        }
      }
      bf16* op = a.out + (long long)m * a.ldo + a.co_off + n;
      if (full && ((a.ldo | a.co_off) & 3) == 0) {
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)apply_act(v[q], a.act);
        *reinterpret_cast<bf16x4*>(op) = o;
      } else {
        for (int q = 0; q < 4; ++q)
          if (n + q < a.Cout) op[q] = (bf16)apply_act(v[q], a.act);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// 1x1 / stride-1 specialisation for shallow K (K = 32*KS <= 192: the MobileNetV2
// expansions and small projections). PMC on the generic kernel above (B=32
// 160->960 expansion): 58 % of wave cycles waiting on memory, ~760 VALU
// instructions per wave for 40 MFMAs. Here every A/B fragment of the whole K is
// issued up front (one memory round trip per wave instead of one per 32-deep
// step), pixel offsets are computed once in 32-bit, and bias comes in as float4.
template <int MT, int NT, int KS>
__global__ __launch_bounds__(256) void conv1x1_kernel(ConvArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = a.B * a.OH * a.OW;
  const int tiles_m = cdiv_dev(M, 32 * MT), tiles_n = cdiv_dev(a.Cout, 32 * NT);
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  const int pix0 = tm * 32 * MT + wm * 16 * MT;
  const int ch0 = tn * 32 * NT + wn * 16 * NT;
  const int r = lane & 15, kq = lane >> 4;
  bf16x8 bfr[KS][MT], afr[KS][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = pix0 + i * 16 + r;
    const bf16* src = a.in + (size_t)(m < M ? m : 0) * a.Cin + kq * 8;
#pragma unroll
    for (int k = 0; k < KS; ++k) bfr[k][i] = m < M ? ld8(src + k * 32) : zero8();
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = ch0 + j * 16 + r;
    const bf16* src = a.w + (size_t)(n < a.Cout ? n : 0) * a.Cin + kq * 8;
#pragma unroll
    for (int k = 0; k < KS; ++k) afr[k][j] = n < a.Cout ? ld8(src + k * 32) : zero8();
  }
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KS; ++k) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[k][j], bfr[k][i], c, 0, 0, 0);
      acc[i][j] = c;
    }
  const int HW = a.OH * a.OW;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = ch0 + j * 16 + kq * 4;
    if (n >= a.Cout) continue;
    const bool full = n + 3 < a.Cout;
    float bv[4];
    if (full) {
      const float4 b4 = *reinterpret_cast<const float4*>(a.bias + n);
      bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[q] = n + q < a.Cout ? a.bias[n + q] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = pix0 + i * 16 + r;
      if (m >= M) continue;
      float v[4] = {acc[i][j][0] + bv[0], acc[i][j][1] + bv[1], acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]};
      if (a.img_bias) {
        const int b = m / HW;
#pragma unroll
        for (int q = 0; q < 4; ++q) if (n + q < a.Cout) v[q] += a.img_bias[(size_t)b * a.Cout + n + q];
      }
      if (a.res) {
        const bf16* rp = a.res + (size_t)m * a.ldr + n;
        if (full && (a.ldr & 3) == 0) {
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(rp);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += (float)rv[q];
        } else {
          for (int q = 0; q < 4; ++q) if (n + q < a.Cout) v[q] += (float)rp[q];
        }
      }
      bf16* op = a.out + (size_t)m * a.ldo + a.co_off + n;
      if (full && ((a.ldo | a.co_off) & 3) == 0) {
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)apply_act(v[q], a.act);
        *reinterpret_cast<bf16x4*>(op) = o;
      } else {
        for (int q = 0; q < 4; ++q)
          if (n + q < a.Cout) op[q] = (bf16)apply_act(v[q], a.act);
      }
    }
  }
}

template <int MT, int NT>
static bool launch_conv1x1(const ConvArgs& a, hipStream_t s) {
  const int M = a.B * a.OH * a.OW;
  const int grid = cdiv(M, 32 * MT) * cdiv(a.Cout, 32 * NT);
  switch (a.Cin / 32) {
#define C1(KS) case KS: hipLaunchKernelGGL((conv1x1_kernel<MT, NT, KS>), dim3(grid), dim3(256), 0, s, a); break;
    C1(1) C1(2) C1(3) C1(4) C1(5) C1(6)
#undef C1
    default: return false;
  }
  check_launch("conv1x1");
  return true;
}

// ---------------------------------------------------------------------------
// LDS-staged variant for the compute-heavy shapes (M = B*OH*OW large).
//
// Block tile: BM = 32*MT pixels x BN = 32*NT output channels, 4 waves (2 x 2),
// wave tile (16*MT) x (16*NT). K is walked in stages of 32*KS elements of one
// tap: every thread loads its 16-byte chunks of the pixel tile (gathered through
// the tap's spatial shift, zero outside the image) and of the weight tile into
// registers, the registers land in an XOR-swizzled LDS image (chunk ^ (row & 7):
// the 16 rows a ds_read_b128 lane group touches spread over 8 bank slots), and
// the next stage's global loads are issued before the current stage's MFMAs so
// their latency hides under the math (one barrier per stage, 2 LDS buffers).
// Taps whose receptive shift puts every pixel of the block tile outside the
// image are skipped block-uniformly.
template <int MT, int NT, int KS>
__global__ __launch_bounds__(256) void conv_gemm_lds_kernel(ConvArgs a) {
  constexpr int BM = 32 * MT, BN = 32 * NT, BKE = 32 * KS;  // BKE: K elements per stage
  constexpr int CPR = BKE / 8;                               // 16-B chunks per row
  constexpr int PCH = BM * CPR / 256, WCH = (BN * CPR + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* sP = reinterpret_cast<bf16*>(smem);                  // [2][BM][BKE]
  bf16* sW = sP + 2 * BM * BKE;                              // [2][BN][BKE]
  int& s_tapmask = *reinterpret_cast<int*>(sW + 2 * BN * BKE);  // one LDS array only

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = a.B * a.OH * a.OW;
  const int tiles_m = cdiv_dev(M, BM), tiles_n = cdiv_dev(a.Cout, BN);
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int taps = a.KH * a.KW;

  // staged pixel rows of this thread
  int rb[PCH], ry[PCH], rx[PCH], rkc[PCH], rrow[PCH];
  bool rv[PCH];
  int tapbits = 0;
#pragma unroll
  for (int i = 0; i < PCH; ++i) {
    const int c = tid + 256 * i;
    rrow[i] = c / CPR;
    rkc[i] = c % CPR;
    const int m = m0 + rrow[i];
    rv[i] = m < M;
    const int mm = rv[i] ? m : 0;
    rb[i] = mm / (a.OH * a.OW);
    const int rem = mm - rb[i] * a.OH * a.OW;
    ry[i] = (rem / a.OW) * a.stride;
    rx[i] = (rem % a.OW) * a.stride;
    if (rv[i]) {
      for (int t = 0; t < taps; ++t) {
        const int iy = ry[i] + (t / a.KW - a.KH / 2) * a.dil;
        const int ix = rx[i] + (t % a.KW - a.KW / 2) * a.dil;
        if (iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW) tapbits |= 1 << t;
      }
    }
  }
  if (tid == 0) s_tapmask = 0;
  __syncthreads();
  if (tapbits) atomicOr(&s_tapmask, tapbits);
  __syncthreads();
  const int tapmask = s_tapmask;

  const int cchunks = cdiv_dev(a.Cin, BKE);
  const int total = taps * cchunks;
  const long long wrow = (long long)taps * a.Cin;

  bf16x8 pr[PCH], wr[WCH];
  auto load = [&](int it) {
    const int t = it / cchunks, c0 = (it % cchunks) * BKE;
    const int dy = (t / a.KW - a.KH / 2) * a.dil, dx = (t % a.KW - a.KW / 2) * a.dil;
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int iy = ry[i] + dy, ix = rx[i] + dx;
      const int c = c0 + rkc[i] * 8;
      const bool ok = rv[i] && c < a.Cin && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
      pr[i] = ok ? ld8(a.in + (((long long)rb[i] * a.IH + iy) * a.IW + ix) * a.Cin + c) : zero8();
    }
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int cidx = tid + 256 * i;
      const int n = cidx / CPR, c = c0 + (cidx % CPR) * 8;
      const bool ok = cidx < BN * CPR && n0 + n < a.Cout && c < a.Cin;
      wr[i] = ok ? ld8(a.w + (long long)(n0 + n) * wrow + (long long)t * a.Cin + c) : zero8();
    }
  };
  auto store = [&](int buf) {
    bf16* P = sP + buf * BM * BKE;
    bf16* Wt = sW + buf * BN * BKE;
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int r = rrow[i];
      st8(P + r * BKE + ((rkc[i] ^ (r & (CPR - 1))) * 8), pr[i]);
    }
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int cidx = tid + 256 * i;
      if (cidx < BN * CPR) {
        const int n = cidx / CPR, kc = cidx % CPR;
        st8(Wt + n * BKE + ((kc ^ (n & (CPR - 1))) * 8), wr[i]);
      }
    }
  };
  auto next_valid = [&](int it) {
    while (it < total && !((tapmask >> (it / cchunks)) & 1)) ++it;
    return it;
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, kq = lane >> 4;
  int it = next_valid(0);
  int buf = 0;
  if (it < total) {
    load(it);
    store(0);
  }
  __syncthreads();
  while (it < total) {
    const int nit = next_valid(it + 1);
    if (nit < total) load(nit);
    const bf16* P = sP + buf * BM * BKE;
    const bf16* Wt = sW + buf * BN * BKE;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 bfr[MT], afr[NT];
      const int kc = ks * 4 + kq;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int r = wm * 16 * MT + i * 16 + r16;
        bfr[i] = ld8(P + r * BKE + ((kc ^ (r & (CPR - 1))) * 8));
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = wn * 16 * NT + j * 16 + r16;
        afr[j] = ld8(Wt + n * BKE + ((kc ^ (n & (CPR - 1))) * 8));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[j], bfr[i], acc[i][j], 0, 0, 0);
    }
    if (nit < total) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
    it = nit;
  }

  // epilogue: lane holds channels n0 + wn*16*NT + j*16 + kq*4 + {0..3} of pixel m
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = m0 + wm * 16 * MT + i * 16 + r16;
    if (m >= M) continue;
    const int b = m / (a.OH * a.OW);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = n0 + wn * 16 * NT + j * 16 + kq * 4;
      if (n >= a.Cout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      const bool full = n + 3 < a.Cout;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (n + q < a.Cout) {
          v[q] += a.bias[n + q];
          if (a.img_bias) v[q] += a.img_bias[(long long)b * a.Cout + n + q];
        }
      }
      if (a.res) {
        const bf16* rp = a.res + (long long)m * a.ldr + n;
        if (full && (a.ldr & 3) == 0) {
          const bf16x4 rv4 = *reinterpret_cast<const bf16x4*>(rp);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += (float)rv4[q];
        } else {
          for (int q = 0; q < 4; ++q) if (n + q < a.Cout) v[q] += (float)rp[q];
        }
      }
      bf16* op = a.out + (long long)m * a.ldo + a.co_off + n;
      if (full && ((a.ldo | a.co_off) & 3) == 0) {
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)apply_act(v[q], a.act);
        *reinterpret_cast<bf16x4*>(op) = o;
      } else {
        for (int q = 0; q < 4; ++q)
          if (n + q < a.Cout) op[q] = (bf16)apply_act(v[q], a.act);
      }
    }
  }
}

static int pick_nt(int Cout);
// ---------------------------------------------------------------------------
// LDS-DMA pipelined variant: operand tiles go global -> LDS with gfx950's
// global_load_lds_dwordx4 (no VGPR staging, no ds_write pass), ST-stage ring with
// ST-1 stages in flight across raw s_barriers and a counted vmcnt, so HBM/MALL
// latency hides behind several K-steps of MFMA even at 1-2 blocks per CU (the
// regime of every deep-K conv here: 128x128 tiles over M = B*33*33 or B*65*65).
// One glds wave-instruction writes 1 KiB = 8 rows x 128 B lane-linearly, so the
// XOR swizzle (phys chunk = logical ^ (row & 7)) is applied on the SOURCE
// address; padded chunks (outside the image, beyond Cin/Cout, M tail) read zeros through
// the buffer descriptor's range check, so the LDS image is always fully written.
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// slices the in-launch split-K combine loads per round trip
constexpr int kInlineKS = 8;

// One BM x BN output tile (tile index bid in row-major (m-tile, n-tile) order) of
// the LDS-DMA conv GEMM; shared by the single-conv kernel and the grouped kernel.
// BK: K depth of one stage (64: 128-byte rows, 8 per glds; 32: 64-byte rows, 16 per
// glds). BK = 32 halves each stage, so the same LDS holds twice the stages: with
// ST = 4 three stages of loads stay in flight across every barrier (the deep-K
// ASPP tiles run at one workgroup per CU, where one stage of lookahead leaves the
// L2/MALL latency exposed).
template <int MT, int NT, int ST, int WM, int WN, int BK = 64>
__device__ __forceinline__ void glds_tile(const ConvArgs& a, const int bid, char* smem, int ks = 1, int kslice = 0,
                                          float* part = nullptr, int* cnt = nullptr) {
  constexpr int NW = WM * WN;                            // waves: WM (pixels) x WN (channels)
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN, ROWB = BK * 2;  // BK bf16 per stage row
  constexpr int CPR = ROWB / 16, RPG = 1024 / ROWB;      // 16-B chunks per row, rows per glds
  constexpr int KS = BK / 32;                            // MFMA k-steps per stage
  static_assert(BK == 64 || BK == 32, "BK 64 or 32");
  constexpr int GA = BM / (RPG * NW), GB = BN / (RPG * NW);  // glds per thread per stage
  static_assert(GA * RPG * NW == BM && GB * RPG * NW == BN, "tile rows must split over the waves");
  constexpr int SB = (BM + BN) * ROWB;
  constexpr int VM_INFLIGHT = (ST - 2) * (GA + GB);
  int* s_tap = reinterpret_cast<int*>(smem + ST * SB);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int r16 = lane & 15, kq = lane >> 4;
  // GEMM rows: output pixels, optionally through a permutation that groups pixels
  // of equal tap validity into whole tiles (dilated ASPP branches: the tile tap
  // mask below then skips every all-padding tap, not only the row-uniform ones)
  const int M = a.perm ? a.Mp : a.B * a.OH * a.OW;
  const int tiles_n = cdiv_dev(a.Cout, BN);
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int taps = a.KH * a.KW;
  const int grow = lane / CPR;                    // row inside the RPG-row group of one glds
  const int lc = (lane % CPR) ^ (grow % CPR);     // logical K-chunk this lane fetches

  int ay[GA], ax[GA], aoff[GA];
  bool av[GA];
  int tapbits = 0;
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int m = m0 + wid * (BM / NW) + i * RPG + grow;
    const int pm = m < M ? (a.perm ? a.perm[m] : m) : -1;
    av[i] = pm >= 0;
    const int mm = av[i] ? pm : 0;
    const int b = mm / (a.OH * a.OW);
    const int rem = mm - b * a.OH * a.OW;
    ay[i] = (rem / a.OW) * a.stride;
    ax[i] = (rem % a.OW) * a.stride;
    aoff[i] = ((b * a.IH + ay[i]) * a.IW + ax[i]) * a.Cin;
    if (av[i]) tapbits |= conv_tap_mask(ay[i], ax[i], a.KH, a.KW, a.dil, a.IH, a.IW);
  }
  unsigned boff2[GB];  // weight row byte offsets, kOOB past Cout
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int n = n0 + wid * (BN / NW) + j * RPG + grow;
    boff2[j] = n < a.Cout ? (unsigned)(n * taps * a.Cin) * 2u : 0x80000000u;
  }
  if (tid == 0) *s_tap = 0;
  __syncthreads();
  if (tapbits) atomicOr(s_tap, tapbits);
  __syncthreads();
  const int tapmask = __builtin_amdgcn_readfirstlane(*s_tap);
  unsigned long long tl = 0;  // live taps, 4 bits each
  int ntap = 0;
  for (int t = 0; t < taps; ++t)
    if ((tapmask >> t) & 1) { tl |= (unsigned long long)t << (4 * ntap); ++ntap; }
  const int cch = cdiv_dev(a.Cin, BK);
  // split-K (small batches: a batch-1 ASPP grid is 40 tiles of up to 45 stages): this block
  // runs stages [s0, s1) of the tile's (tap, channel-chunk) sequence
  const int s0 = kslice * (ntap * cch) / ks, s1 = (kslice + 1) * (ntap * cch) / ks;
  const int total = s1 - s0;

  int is_tap = s0 / cch, is_c = s0 - (s0 / cch) * cch;  // issue cursor
  // per-tap state of the cursor, recomputed only when it moves to the next tap: the rows'
  // source offsets (element index of channel 0 for this tap, -1 = padding -> zero page) and
  // the tap's weight offset. Round 2 recomputed the bounds and offsets for every 64-channel
  // stage: ~135 VALU + ~155 SALU per wave and stage against 32 MFMAs (PMC of the 16-wave
  // grouped ASPP tile, profiles/r3_step_pmc.txt)
  // Round 5: the rows arrive through buffer_load ... lds on range-checked descriptors (the
  // int8 kernel's form): a padding row's byte offset carries bit 31, past the descriptor's
  // end, and the hardware writes zeros -- no zero-page pointer selects or 64-bit address math.
  constexpr unsigned kOOB = 0x80000000u;
  const auto rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.in), 0,
                                                     (int)((long long)a.B * a.IH * a.IW * a.Cin * 2), 0x00020000);
  const auto rwt = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.w), 0,
                                                     (int)((long long)a.Cout * taps * a.Cin * 2), 0x00020000);
  unsigned abyte[GA];  // this tap's row byte offsets (channel 0), kOOB for padding
  unsigned wbyte = 0;
  auto set_tap = [&]() {
    const int t = (int)((tl >> (4 * is_tap)) & 15);
    const int dy = (t / a.KW - a.KH / 2) * a.dil, dx = (t % a.KW - a.KW / 2) * a.dil;
    const int doff = (dy * a.IW + dx) * a.Cin;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int iy = ay[i] + dy, ix = ax[i] + dx;
      const bool ok = av[i] && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
      abyte[i] = ok ? (unsigned)(aoff[i] + doff) * 2u : kOOB;
    }
    wbyte = (unsigned)(t * a.Cin) * 2u;
  };
  if (total > 0) set_tap();
  const int cin_left = a.Cin - lc * 8;  // this lane's 16-byte chunk exists while is_c * BK < cin_left
  auto issue = [&](int stage) {
    const int cb = is_c * BK;
    const unsigned cbad = (unsigned)(cin_left - cb - 1) & kOOB;
    const unsigned cbyte = (unsigned)(cb + lc * 8) * 2u;
    char* sA = smem + stage * SB;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const unsigned vo = (abyte[i] + cbyte) | cbad;  // (a named offset: the host pass rejects the inline form)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_ptr_t)(sA + (wid * (BM / NW) + i * RPG) * ROWB), 16, vo, 0, 0, 0);
    }
    char* sB = sA + BM * ROWB;
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const unsigned vo = (boff2[j] + wbyte + cbyte) | cbad;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwt, (lds_ptr_t)(sB + (wid * (BN / NW) + j * RPG) * ROWB), 16, vo, 0, 0, 0);
    }
    if (++is_c == cch) {
      is_c = 0;
      if (++is_tap < ntap) set_tap();
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < ST - 1; ++s)
    if (s < total) issue(s);
  for (int k = 0; k < total; ++k) {
    if (k + ST - 2 < total) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_INFLIGHT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (k + ST - 1 < total) issue((k + ST - 1) % ST);
    const char* sA = smem + (k % ST) * SB;
    const char* sB = sA + BM * ROWB;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int kc = ks * 4 + kq;
      bf16x8 bfr[MT], afr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int r = wm * 16 * MT + i * 16 + r16;
        bfr[i] = *reinterpret_cast<const bf16x8*>(sA + r * ROWB + ((kc ^ (r % CPR)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = wn * 16 * NT + j * 16 + r16;
        afr[j] = *reinterpret_cast<const bf16x8*>(sB + n * ROWB + ((kc ^ (n % CPR)) << 4));
      }
      // T5: raise this wave's issue priority over the MFMA cluster, so the SIMD's
      // other wave (2 per SIMD at 8 waves) does not interleave its LDS reads into it
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[j], bfr[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  if (part) {  // split-K: fp32 partial of this slice, bias / activation in the combine
    const size_t slab = (size_t)a.B * a.OH * a.OW * a.ldo;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int mg = m0 + wm * 16 * MT + i * 16 + r16;
      if (mg >= M) continue;
      const int m = a.perm ? a.perm[mg] : mg;
      if (m < 0) continue;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n0 + wn * 16 * NT + j * 16 + kq * 4;
        if (n < a.Cout) *reinterpret_cast<f32x4*>(part + kslice * slab + (size_t)m * a.ldo + a.co_off + n) = acc[i][j];
      }
    }
    if (cnt) {
      // in-launch combine (the split-K recipe of cdna_hip_programming.md): drain, release,
      // draw a ticket; the tile's last arriving slice acquires, resets the ticket and sums
      // the ks slabs in slice order (+ bias, activation) into the bf16 output
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // every wave's stores drained, every LDS read of the K loop done
      int* s_flag = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int t = __hip_atomic_fetch_add(cnt + bid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = t == ks - 1;
        if (last) {
          __hip_atomic_store(cnt + bid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *s_flag = last;
      }
      __syncthreads();
      if (*reinterpret_cast<volatile int*>(s_flag)) {
        constexpr int NTH = 64 * NW, Q = BN / 4;
        for (int idx = tid; idx < BM * Q; idx += NTH) {
          const int r = idx / Q, n = n0 + (idx - r * Q) * 4;
          const int mg = m0 + r;
          if (mg >= M || n >= a.Cout) continue;
          const int m = a.perm ? a.perm[mg] : mg;
          if (m < 0) continue;
          const float* q = part + (size_t)m * a.ldo + a.co_off + n;
          f32x4 v = *reinterpret_cast<const f32x4*>(a.bias + n);
          // the slices' loads issued kInlineKS at a time before their adds (one L2 round
          // trip per group, not one per slice); slices past ks re-read the last one and are
          // not added; order sl = 0..ks-1
          for (int s0 = 0; s0 < ks; s0 += kInlineKS) {
            f32x4 pv[kInlineKS];
#pragma unroll
            for (int sl = 0; sl < kInlineKS; ++sl)
              pv[sl] = *reinterpret_cast<const f32x4*>(q + (size_t)(s0 + sl < ks ? s0 + sl : ks - 1) * slab);
#pragma unroll
            for (int sl = 0; sl < kInlineKS; ++sl)
              if (s0 + sl < ks) v += pv[sl];
          }
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (bf16)apply_act(v[e], a.act);
          *reinterpret_cast<bf16x4*>(a.out + (size_t)m * a.ldo + a.co_off + n) = o;
        }
      }
    }
    return;
  }
  // the lane's 4 output channels of each 16-channel subtile are the same for every pixel
  // subtile: their bias is loaded once (one 16-byte load per j, not 4 x MT scalar loads)
  f32x4 bj[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = n0 + wn * 16 * NT + j * 16 + kq * 4;
    if (n + 3 < a.Cout) {
      bj[j] = *reinterpret_cast<const f32x4*>(a.bias + n);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) bj[j][q] = n + q < a.Cout ? a.bias[n + q] : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int mg = m0 + wm * 16 * MT + i * 16 + r16;
    if (mg >= M) continue;
    const int m = a.perm ? a.perm[mg] : mg;
    if (m < 0) continue;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = n0 + wn * 16 * NT + j * 16 + kq * 4;
      if (n >= a.Cout) continue;
      float v[4] = {acc[i][j][0] + bj[j][0], acc[i][j][1] + bj[j][1], acc[i][j][2] + bj[j][2],
                    acc[i][j][3] + bj[j][3]};
      const bool full = n + 3 < a.Cout;
      if (a.img_bias) {
        const int b = m / (a.OH * a.OW);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (n + q < a.Cout) v[q] += a.img_bias[(long long)b * a.Cout + n + q];
      }
      if (a.res) {
        const bf16* rp = a.res + (long long)m * a.ldr + n;
        if (full && (a.ldr & 3) == 0) {
          const bf16x4 rv4 = *reinterpret_cast<const bf16x4*>(rp);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += (float)rv4[q];
        } else {
          for (int q = 0; q < 4; ++q) if (n + q < a.Cout) v[q] += (float)rp[q];
        }
      }
      bf16* op = a.out + (long long)m * a.ldo + a.co_off + n;
      if (full && ((a.ldo | a.co_off) & 3) == 0) {
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)apply_act(v[q], a.act);
        *reinterpret_cast<bf16x4*>(op) = o;
      } else {
        for (int q = 0; q < 4; ++q)
          if (n + q < a.Cout) op[q] = (bf16)apply_act(v[q], a.act);
      }
    }
  }
}

template <int MT, int NT, int ST, int WM = 2, int WN = 2>
__global__ __launch_bounds__(64 * WM * WN) void conv_glds_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const int M = a.perm ? a.Mp : a.B * a.OH * a.OW;
  const int tiles = cdiv_dev(M, BM) * cdiv_dev(a.Cout, BN);
  glds_tile<MT, NT, ST, WM, WN>(a, xcd_remap(blockIdx.x, tiles), smem);
}

// Grouped launch: up to kMaxConvGroup independent convs (the ASPP branches, which
// read the same input and write disjoint channel slices of one concat buffer) in
// ONE grid. Block i runs tile order[i] = (group << 24) | tile; the host sorts the
// tiles by live-tap work, heaviest first (LPT), so the per-branch grids that left
// half the CUs idle (137 256x256 tiles of a 34848 x 256 GEMM on 256 CUs) become
// one balanced grid with no per-branch tail.
template <int MT, int NT, int ST, int WM = 2, int WN = 2, int BK = 64>
__global__ __launch_bounds__(64 * WM * WN) void conv_glds_group_kernel(ConvGroupArgs ga) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int e = __builtin_amdgcn_readfirstlane(ga.order[blockIdx.x]);
  const int t = e & 0xfffff, ksl = (e >> 20) & 15;
  switch (e >> 24) {  // constant indices: each arm reads its ConvArgs straight from kernarg
    case 0: glds_tile<MT, NT, ST, WM, WN, BK>(ga.g[0], t, smem, ga.ks, ksl, ga.part, ga.cnt); break;
    case 1: glds_tile<MT, NT, ST, WM, WN, BK>(ga.g[1], t, smem, ga.ks, ksl, ga.part,
                                              ga.cnt ? ga.cnt + ga.cnt_stride : nullptr); break;
    case 2: glds_tile<MT, NT, ST, WM, WN, BK>(ga.g[2], t, smem, ga.ks, ksl, ga.part,
                                              ga.cnt ? ga.cnt + 2 * ga.cnt_stride : nullptr); break;
    default: glds_tile<MT, NT, ST, WM, WN, BK>(ga.g[3], t, smem, ga.ks, ksl, ga.part,
                                               ga.cnt ? ga.cnt + 3 * ga.cnt_stride : nullptr); break;
  }
}

template <int MT, int NT, int ST, int WM = 2, int WN = 2, int BK = 64>
static void launch_conv_glds_group(const ConvGroupArgs& ga, int nblocks, hipStream_t s) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const size_t lds = (size_t)ST * (BM + BN) * BK * 2 + 16;
  static_assert((size_t)ST * (BM + BN) * BK * 2 + 16 <= 160 * 1024, "LDS ring too large");
  static bool attr_set = false;
  if (!attr_set) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_glds_group_kernel<MT, NT, ST, WM, WN, BK>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "conv_glds_group attr");
    attr_set = true;
  }
  hipLaunchKernelGGL((conv_glds_group_kernel<MT, NT, ST, WM, WN, BK>), dim3(nblocks),
                     dim3(64 * WM * WN), lds, s, ga);
  check_launch("conv_glds_group");
}

template <int MT, int NT, int ST, int WM = 2, int WN = 2>
static void launch_conv_glds(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const int M = a.perm ? a.Mp : a.B * a.OH * a.OW;
  const int grid = cdiv(M, BM) * cdiv(a.Cout, BN);
  const size_t lds = (size_t)ST * (BM + BN) * 128 + 16;
  static bool attr_set = false;
  if (!attr_set) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_glds_kernel<MT, NT, ST, WM, WN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "conv_glds attr");
    attr_set = true;
  }
  hipLaunchKernelGGL((conv_glds_kernel<MT, NT, ST, WM, WN>), dim3(grid), dim3(64 * WM * WN), lds, s, a);
  check_launch("conv_glds");
}

template <int ST>
static void dispatch_glds(const ConvArgs& a, hipStream_t s) {
  switch (pick_nt(a.Cout)) {
    case 1: launch_conv_glds<4, 1, ST>(a, s); break;
    case 2: launch_conv_glds<4, 2, ST>(a, s); break;
    case 3: launch_conv_glds<4, 3, ST>(a, s); break;
    case 4: launch_conv_glds<4, 4, ST>(a, s); break;
    case 5: launch_conv_glds<4, 5, ST>(a, s); break;
    default: launch_conv_glds<4, 6, ST>(a, s); break;
  }
}

template <int MT, int NT, int KS>
static void launch_conv_lds(const ConvArgs& a, hipStream_t s) {
  const int M = a.B * a.OH * a.OW;
  const int grid = cdiv(M, 32 * MT) * cdiv(a.Cout, 32 * NT);
  const size_t lds = (size_t)2 * (32 * MT + 32 * NT) * 32 * KS * sizeof(bf16) + 16;
  hipLaunchKernelGGL((conv_gemm_lds_kernel<MT, NT, KS>), dim3(grid), dim3(256), lds, s, a);
  check_launch("conv_gemm_lds");
}

// channel-tile choice: NT in 1..6 (BN = 32*NT) minimising padded columns
static int pick_nt(int Cout) {
  if (Cout <= 192) return (Cout + 31) / 32;
  int best = 4, waste = 1 << 30;
  for (int nt = 6; nt >= 4; --nt) {
    const int w = cdiv(Cout, 32 * nt) * 32 * nt - Cout;
    if (w < waste) { waste = w; best = nt; }
  }
  return best;
}

template <int KS>
static void dispatch_lds(const ConvArgs& a, hipStream_t s) {
  switch (pick_nt(a.Cout)) {
    case 1: launch_conv_lds<4, 1, KS>(a, s); break;
    case 2: launch_conv_lds<4, 2, KS>(a, s); break;
    case 3: launch_conv_lds<4, 3, KS>(a, s); break;
    case 4: launch_conv_lds<4, 4, KS>(a, s); break;
    case 5: launch_conv_lds<4, 5, KS>(a, s); break;
    default: launch_conv_lds<4, 6, KS>(a, s); break;
  }
}

template <int MT, int NT>
static void launch_conv(const ConvArgs& a, hipStream_t s) {
  const int M = a.B * a.OH * a.OW;
  const int grid = cdiv(M, 32 * MT) * cdiv(a.Cout, 32 * NT);
  hipLaunchKernelGGL((conv_gemm_kernel<MT, NT>), dim3(grid), dim3(256), 0, s, a);
  check_launch("conv_gemm");
}

void conv_gemm(const ConvParams& p, hipStream_t s) {
  if (p.Cin % 8 != 0) throw std::invalid_argument("conv_gemm: Cin must be a multiple of 8");
  if (p.co_off % 1 != 0 || p.ldo < p.co_off + p.Cout) throw std::invalid_argument("conv_gemm: bad ldo/co_off");
  if (p.res && p.ldr < p.Cout) throw std::invalid_argument("conv_gemm: bad ldr");
  ConvArgs a{p.in, p.w, p.bias, p.img_bias, p.res, p.out, p.B, p.IH, p.IW, p.Cin, p.OH, p.OW,
             p.Cout, p.KH, p.KW, p.stride, p.dil, p.ldo, p.co_off, p.ldr, p.act, p.perm, p.Mp};
  const long long M = (long long)p.B * p.OH * p.OW;
  const long long tiles = (M + 127) / 128 * cdiv(p.Cout, 32 * pick_nt(p.Cout));
  const long long K = (long long)p.KH * p.KW * p.Cin;
  // auto: LDS-DMA 2-stage for deep K on grids that fill the chip (scripts/bench_conv.py
  // on MI355X: 1.2-1.9x the register-staged LDS kernel from K = 256 up; shallow-K
  // layers are output-write-bound and stay on the register-fed kernel)
  // 32-bit buffer byte offsets below 2^31 (bf16: 2^30 elements), <= 16 taps in the tap list
  const bool glds_ok = (long long)p.B * p.IH * p.IW * p.Cin < (1LL << 30) &&
                       (long long)p.Cout * K < (1LL << 30) && p.KH * p.KW <= 16;
  int variant = p.variant;
  if (variant == 0) variant = (tiles >= 128 && K >= 256) ? (glds_ok ? 4 : 2) : 1;
  if (p.perm && (variant < 3 || variant == 7 || variant > 10 || !glds_ok))
    throw std::invalid_argument("conv_gemm: a pixel permutation needs an LDS-DMA variant (3-6)");
  if (variant == 3 || variant == 4) {
    if (!glds_ok) throw std::invalid_argument("conv_gemm glds: tensor too large for 32-bit offsets or > 16 taps");
    if (variant == 3) dispatch_glds<3>(a, s);
    else dispatch_glds<2>(a, s);
    return;
  }
  if (variant >= 8 && variant <= 10) {
    // deeper rings (ST = 3/4 stages, 2-3 K-steps in flight) at one workgroup per CU:
    // 8: 128 x 256, 8 waves (2 per SIMD), ST 3 -- ASPP-class N = 256
    // 9: 64 x (32*nt), 4 waves, ST 4 -- the 33x33 projections (N = 96..320)
    // 10: 128 x 128, 4 waves, ST 4
    if (!glds_ok) throw std::invalid_argument("conv_gemm glds: tensor too large for 32-bit offsets or > 16 taps");
    if (variant == 8) launch_conv_glds<4, 4, 3, 2, 4>(a, s);
    else if (variant == 10) launch_conv_glds<4, 4, 4, 2, 2>(a, s);
    else switch (pick_nt(p.Cout)) {
      case 1: launch_conv_glds<2, 1, 4, 2, 2>(a, s); break;
      case 2: launch_conv_glds<2, 2, 4, 2, 2>(a, s); break;
      case 3: launch_conv_glds<2, 3, 4, 2, 2>(a, s); break;
      case 4: launch_conv_glds<2, 4, 4, 2, 2>(a, s); break;
      case 5: launch_conv_glds<2, 5, 4, 2, 2>(a, s); break;
      default: launch_conv_glds<2, 6, 4, 2, 2>(a, s); break;
    }
    return;
  }
  if (variant == 5 || variant == 6) {
    // wide tiles, 8 waves (2 x 4): 128 x 256 (5) / 256 x 256 (6) -- the A (pixel)
    // tile is fetched once for all 256 output channels of the ASPP-class layers,
    // fewer L2->LDS bytes per MAC where per-CU fill bandwidth is the limit
    if (!glds_ok) throw std::invalid_argument("conv_gemm glds: tensor too large for 32-bit offsets or > 16 taps");
    if (variant == 5) launch_conv_glds<4, 4, 2, 2, 4>(a, s);
    else launch_conv_glds<8, 4, 2, 2, 4>(a, s);
    return;
  }
  if (variant == 2) {
    // LDS-staged MFMA path: deep K (ASPP atrous 2880, projections 576-1024) and
    // enough 128-pixel tiles to fill the chip. Shallow-K layers are write-bound
    // and measured faster on the register-fed kernel (rocprof, B=32 MNv2).
    if (p.Cin <= 32) dispatch_lds<1>(a, s);
    else dispatch_lds<2>(a, s);
    return;
  }
  // shallow-K 1x1 stride-1 layers: all-K-up-front specialisation
  const bool k1 = p.KH == 1 && p.KW == 1 && p.stride == 1 && p.OH == p.IH && p.OW == p.IW &&
                  p.Cin % 32 == 0 && p.Cin <= 192 && M * (long long)p.Cin < (1LL << 31);
  if (k1 && (variant == 7 || p.variant == 0)) {
    bool ok;
    if (p.Cout <= 32) ok = launch_conv1x1<4, 1>(a, s);
    else if (p.Cout <= 64 || M < 8192) ok = launch_conv1x1<2, 2>(a, s);
    else ok = launch_conv1x1<2, 4>(a, s);
    if (ok) return;
  }
  // direct path (small M, e.g. batch-1 33x33 maps): smaller tiles, more blocks
  if (p.Cout <= 32) {
    launch_conv<4, 1>(a, s);  // 128 px x 32 ch
  } else if (p.Cout <= 64 || M < 8192) {
    launch_conv<2, 2>(a, s);  // 64 px x 64 ch
  } else {
    launch_conv<2, 4>(a, s);  // 64 px x 128 ch
  }
}

static ConvArgs to_args(const ConvParams& p) {
  return ConvArgs{p.in, p.w, p.bias, p.img_bias, p.res, p.out, p.B, p.IH, p.IW, p.Cin, p.OH, p.OW,
                  p.Cout, p.KH, p.KW, p.stride, p.dil, p.ldo, p.co_off, p.ldr, p.act, p.perm, p.Mp};
}

void conv_gemm_grouped(const ConvParams* ps, int n, const int* order, int nblocks, int variant,
                       hipStream_t s, int ks, float* part, int* cnt, int cnt_stride) {
  if (n < 1 || n > kMaxConvGroup) throw std::invalid_argument("conv_gemm_grouped: 1..4 convs");
  if (!order || nblocks < 1) throw std::invalid_argument("conv_gemm_grouped: empty tile order");
  if (ks < 1 || ks > 16 || (ks > 1 && part == nullptr))
    throw std::invalid_argument("conv_gemm_grouped: ks in [1, 16], a partials buffer for ks > 1");
  if (ks > 1)
    for (int i = 0; i < n; ++i)
      if (ps[i].ldo != ps[0].ldo || ps[i].Cout % 4 || (ps[i].ldo | ps[i].co_off) % 4)
        throw std::invalid_argument("conv_gemm_grouped: split-K needs one ldo and 4-aligned channels");
  ConvGroupArgs ga{};
  ga.ks = ks;
  ga.part = ks > 1 ? part : nullptr;
  ga.cnt = ks > 1 ? cnt : nullptr;
  ga.cnt_stride = cnt_stride;
  for (int i = 0; i < kMaxConvGroup; ++i) {
    const ConvParams& p = ps[i < n ? i : 0];
    if (p.Cin % 8 != 0 || p.KH * p.KW > 16 || p.Cout != ps[0].Cout)
      throw std::invalid_argument("conv_gemm_grouped: Cin % 8, <= 16 taps and one Cout required");
    if ((long long)p.B * p.IH * p.IW * p.Cin >= (1LL << 30) ||
        (long long)p.Cout * p.KH * p.KW * p.Cin >= (1LL << 30))
      throw std::invalid_argument("conv_gemm_grouped: tensor too large for 32-bit byte offsets");
    ga.g[i] = to_args(p);
  }
  ga.order = order;
  switch (variant) {
    case 5: launch_conv_glds_group<4, 4, 2, 2, 4>(ga, nblocks, s); break;   // 128 x 256, 8 waves
    case 6: launch_conv_glds_group<8, 4, 2, 2, 4>(ga, nblocks, s); break;   // 256 x 256, 8 waves
    case 8: launch_conv_glds_group<4, 4, 3, 2, 4>(ga, nblocks, s); break;   // 128 x 256, 3 stages
    case 10: launch_conv_glds_group<4, 4, 4, 2, 2>(ga, nblocks, s); break;  // 128 x 128, 4 stages
    case 11: launch_conv_glds_group<4, 4, 2, 2, 2>(ga, nblocks, s); break;  // 128 x 128, 2 stages
    // 32-deep stages, 3 in flight
    case 12: launch_conv_glds_group<8, 4, 4, 2, 4, 32>(ga, nblocks, s); break;  // 256 x 256
    case 13: launch_conv_glds_group<4, 4, 4, 2, 4, 32>(ga, nblocks, s); break;  // 128 x 256
    case 14: launch_conv_glds_group<8, 4, 3, 2, 4, 32>(ga, nblocks, s); break;  // 256 x 256, 3 stages
    // 16 waves (4 per SIMD, 64 x 64 per wave): twice the waves of v6 to cover the LDS-DMA
    // and LDS latency of the 1-workgroup-per-CU 256 x 256 tiles (MFMA busy ~23 % in v6)
    case 15: launch_conv_glds_group<4, 4, 2, 4, 4>(ga, nblocks, s); break;      // 256 x 256
    case 16: launch_conv_glds_group<4, 4, 4, 4, 4, 32>(ga, nblocks, s); break;  // 256 x 256, 32-deep
    // 16 waves on half-size tiles (32 x 64 / 64 x 32 per wave): twice the tiles, so the LPT
    // grid's last round (548 tiles of up to 9 taps on 256 CUs at 256 x 256) is finer
    case 17: launch_conv_glds_group<2, 4, 2, 4, 4>(ga, nblocks, s); break;      // 128 x 256
    case 18: launch_conv_glds_group<4, 2, 2, 4, 4>(ga, nblocks, s); break;      // 256 x 128
    default: throw std::invalid_argument("conv_gemm_grouped: variant must be 5, 6, 8, 10-18");
  }
}

}  // namespace ssa
