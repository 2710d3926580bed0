// Row-streaming stem + MobileNetV2 block 0 for gfx950 (the network's first two layers at
// 513^2: 3x3 s2 conv 3 -> 32 + relu6 on the letterboxed camera frame, then block 0 =
// depthwise 3x3 on the 32 stem channels + relu6, projection 32 -> 16).
//
// Round 1-3 ran this as 2-D tiles (stem_block0_kernel, fused_ir.hip): per 16x16 output
// tile the stem was recomputed over an 18x18 halo (1.27x) from a 35x35 gather of
// letterboxed camera pixels (4.8 LUT-chained gathers per output pixel), behind two
// workgroup barriers, and the kernel was VALU- and latency-bound: 100 us per 32 frames in
// the step trace for a ~20 us memory floor (VERDICT r3 Weak #1; PMC ~950 VALU per wave).
//
// Here a workgroup owns R output rows x TW columns and streams down the stem rows:
//   * every model-input pixel of the band is gathered ONCE (camera bytes through the
//     letterbox LUTs, prefetched PD steps ahead into registers, normalised to bf16 RGB0
//     in a 6-row LDS ring);
//   * every stem pixel is computed ONCE (no vertical halo inside the band): 3 MFMAs
//     16x16x16 bf16 per 16 pixels x 16 channels, K = 12 taps x RGB0 (the 4 channels of
//     one input pixel are one 8-byte LDS read), + bias, relu6 -> fp16 stem row in LDS;
//   * the block-0 depthwise accumulates per stem row into register-resident fp16 sums of
//     the 3 output rows that row feeds (bias first, taps in ky-major order: the exact
//     arithmetic of stem_block0_kernel), and a completed row goes straight from registers
//     into the projection MFMA (lane = 8 channels of one pixel = its B fragment).
// One step = one stem row, ONE barrier: [gather next rows | stem row -> S[t & 1]] A
// [depthwise, projection, store from S[t & 1]]. The stem row buffer is double-buffered, so
// the next step's stem (other buffer) may start while a slower wave still runs this step's
// depthwise -- the round-4 form had a second barrier per step for that (86 barriers per
// band of 41 rows, each a full drain of a latency-bound 4-wave workgroup). Ring-row reuse
// with one barrier: step t writes input rows 2t+3, 2t+4 and reads 2t .. 2t+2 (6-row ring);
// the rows step t+1 overwrites (2t-1, 2t) were last read by stem t-1, before barrier t-1.
// Weights live in VGPRs. Output: [B, 257, 257, 16] bf16 (block 1's input). Reference parity: the Edge TPU model's first layers
// (/root/reference/sem_seg_server.py:151-162: BGR->RGB, NEAREST letterbox, quantised input).
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

typedef _Float16 f16;
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

struct StemBandArgs {
  const uint8_t* frames; const int32_t* lut_x; const int32_t* lut_y;
  const bf16* ws; const float* bs; const f16* wd; const f16* bd; const f16* wp; const float* bp;
  bf16* out;
  int B, Hc, Wc, H, W, SH, SW, R, nbx, nby, TW;
};

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

constexpr int kSP = 80;  // stem-row entry pitch (B): 32 fp16 + 16 B pad (odd multiple of 16 B)

// NW waves = column groups of 16 stem columns (the band's TW + 2 stem columns);
// GPX input pixels per lane per gathered row pair
template <int NW, int GPX, bool ONEB>
__global__ __launch_bounds__(64 * NW) void stem_band_kernel(StemBandArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int U = 3;   // step unroll: static D-slot / ring / prefetch roles
  constexpr int PD = 3;  // row pairs prefetched ahead (registers)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;

  int blk = blockIdx.x;
  const int bx = blk % a.nbx;
  blk /= a.nbx;
  const int by = blk % a.nby;
  const int b = blk / a.nby;
  const int x0 = bx * a.TW, y0 = by * a.R, y1 = min(y0 + a.R, a.SH);
  const int twv = min(a.TW, a.SW - x0);
  const int NSC = twv + 2;            // stem columns: global x0 - 1 .. x0 + twv
  const int NIC = 2 * NSC + 1;        // input columns: global 2 x0 - 3 .. 2 (x0 + twv) + 1
  const int ixb = 2 * x0 - 3;
  const int rbase = 2 * y0 - 3;       // global input row of ring row 0 (stem row y0 - 1 reads 2y0-3..2y0-1)
  const int n_st = y1 - y0 + 2;       // stem rows y0 - 1 .. y1
  const int n_rows = 2 * n_st + 1;    // input rows the band reads

  // LDS: [IN ring 6 rows][NIC][8 B] | [S rows 2 x NSC x 80 B] | [lut_y of the band's rows]
  bf16* IN = reinterpret_cast<bf16*>(smem);
  const int in_row = NIC * 4;  // elements per ring row
  char* S2 = smem + (size_t)6 * NIC * 8;
  const int s_bytes = NSC * kSP;
  int* sly = reinterpret_cast<int*>(S2 + (size_t)2 * s_bytes);
  for (int i = tid; i < n_rows; i += NT) {
    const int r = rbase + i;
    sly[i] = (r >= 0 && r < a.H) ? a.lut_y[r] : -2;  // -2: outside the model input (conv zero pad)
  }

  // ---- weights -> VGPRs
  s16x4 wst[2][3];
  f32x4 bst[2];
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
    for (int m = 0; m < 3; ++m)
      wst[sub][m] = *reinterpret_cast<const s16x4*>(a.ws + (size_t)(sub * 16 + r16) * 48 + m * 16 + kq * 4);
    bst[sub] = *reinterpret_cast<const f32x4*>(a.bs + sub * 16 + kq * 4);
  }
  f16x8 wdv[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) wdv[tap] = *reinterpret_cast<const f16x8*>(a.wd + tap * 32 + kq * 8);
  const f16x8 bdv = *reinterpret_cast<const f16x8*>(a.bd + kq * 8);
  const f16x8 af = *reinterpret_cast<const f16x8*>(a.wp + (size_t)r16 * 32 + kq * 8);
  const f32x4 bpv = *reinterpret_cast<const f32x4*>(a.bp + kq * 4);

  // ---- gather lanes: pixel p = tid + u * NT of a row pair -> (row k, local input col i)
  const uint8_t* fb = a.frames + (size_t)b * a.Hc * a.Wc * 3;
  int gk[GPX], gi[GPX], gsx[GPX];  // row in pair, local col, camera col (-1 pad, -2 outside)
#pragma unroll
  for (int u = 0; u < GPX; ++u) {
    const int p = tid + u * NT;
    const bool live = p < 2 * NIC;
    gk[u] = live ? p / NIC : 2;  // 2: no pixel
    gi[u] = live ? p - gk[u] * NIC : 0;
    const int x = ixb + gi[u];
    gsx[u] = (live && x >= 0 && x < a.W) ? a.lut_x[x] : -2;
  }
  __syncthreads();  // sly visible

  // camera bytes of one pixel: -> bf16 RGB0 (x / 127.5 - 1, BGR -> RGB; -1 letterbox pad,
  // 0 outside the model input)
  struct Px { uint32_t c0, c1, c2; int kind; };
  // branch-free: every lane loads a (clamped) pixel, the kind selects at store time (a
  // conditional load makes the compiler wait for it right away)
  auto fetch_px = [&](int rel_row, int u) -> Px {
    const int sy = sly[min(rel_row, n_rows - 1)];
    const int sx = gsx[u];
    Px v;
    v.kind = (gk[u] > 1 || rel_row >= n_rows || sy == -2 || sx == -2) ? -2 : (sy < 0 || sx < 0) ? -1 : 0;
    // 32-bit byte offset from the uniform frame base (a frame is < 4 GiB): SGPR base +
    // VGPR offset addressing, no 64-bit multiply-add per pixel
    const uint8_t* px = fb + (unsigned)((max(sy, 0) * a.Wc + max(sx, 0)) * 3);
    v.c0 = px[0]; v.c1 = px[1]; v.c2 = px[2];
    return v;
  };
  // off: the pixel's element offset in the ring (-1: ring row rel_row % 6 computed here)
  auto store_px = [&](int rel_row, int u, const Px& v, int off = -1) {
    if (gk[u] > 1 || rel_row >= n_rows) return;
    float rgb[3] = {0.f, 0.f, 0.f};
    if (v.kind == 0) {
      rgb[0] = v.c2 * (1.f / 127.5f) - 1.f;
      rgb[1] = v.c1 * (1.f / 127.5f) - 1.f;
      rgb[2] = v.c0 * (1.f / 127.5f) - 1.f;
    } else if (v.kind == -1) {
      rgb[0] = rgb[1] = rgb[2] = -1.f;
    }
    const bf16x4 o = {(bf16)rgb[0], (bf16)rgb[1], (bf16)rgb[2], (bf16)0.f};
    *reinterpret_cast<bf16x4*>(IN + (off >= 0 ? off : (rel_row % 6) * in_row + gi[u] * 4)) = o;
  };
  // row pair q = ring rows 2q + 1, 2q + 2 (step q's new rows; step 0 also reads row 0)
  Px xr[PD][GPX];
  // prologue: rows 0, 1, 2 now; pairs 1..PD in flight
  {
    Px r0[GPX], p0[GPX];
#pragma unroll
    for (int u = 0; u < GPX; ++u) {
      r0[u] = fetch_px(gk[u], u);          // rows 0 and 1 (k = 0, 1)
      p0[u] = fetch_px(2 + gk[u], u);      // rows 2 and 3 (row 3 = pair 1's first row)
    }
#pragma unroll
    for (int u = 0; u < GPX; ++u) {
      store_px(gk[u], u, r0[u]);
      if (gk[u] == 0) store_px(2, u, p0[u]);  // row 2 (pair 0's second row)
    }
  }
#pragma unroll
  for (int q = 1; q <= PD; ++q)
#pragma unroll
    for (int u = 0; u < GPX; ++u) xr[q % PD][u] = fetch_px(2 * q + 1 + gk[u], u);

  // ---- this lane's stem column (stem phase) and output column (depthwise phase)
  const int sj = g * 16 + r16;                // local stem column
  const int sxg = x0 - 1 + sj;                // global stem column
  const bool sin_x = sj < NSC && sxg >= 0 && sxg < a.SW;
  const int sjc = sj < NSC ? sj : 0;
  int toff[3];  // this lane's tap (m*4 + kq) as an element offset: ring-row delta, column
  int tky[3];   // (taps 9-11 pad the last fragment: zero weights, they read tap 0's pixel, so
                // the three fragment reads are unconditional and issue back to back)
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int tp = m * 4 + kq;
    tky[m] = tp < 9 ? tp / 3 : 0;
    toff[m] = (2 * sjc + (tp < 9 ? tp % 3 : 0)) * 4;
  }
  // ring-row offsets by step phase: the loop's t0 is a multiple of U = 3, so the ring row
  // (2t + k) % 6 of step t = t0 + ph is (2 ph + k) % 6 -- static per phase; precomputed here
  // instead of an integer modulo per tap and step (3 stem reads + the gathered rows' stores:
  // ~40 of the step's ~160 VALU)
  static_assert(U == 3, "ring offsets assume the 3-step unroll (2 U == the 6-row ring)");
  int sro[U][3];  // stem fragment reads: (2 ph + tky[m]) % 6 ring row, + toff
  int sto[U][GPX];  // gathered-row stores of step ph (rows 2 (t + 1) + 1 + gk): ring row, + column
#pragma unroll
  for (int ph = 0; ph < U; ++ph) {
#pragma unroll
    for (int m = 0; m < 3; ++m) sro[ph][m] = ((2 * ph + tky[m]) % 6) * in_row + toff[m];
#pragma unroll
    for (int u = 0; u < GPX; ++u) sto[ph][u] = ((2 * ph + 3 + gk[u]) % 6) * in_row + gi[u] * 4;
  }
  const int xl = g * 16 + r16;                // local output column (reads stem cols xl..xl+2)
  const bool xv = xl < twv;
  const int xc = xv ? xl : 0;
  // ReLU6 as a [0, 1] clamp (stem / 6, depthwise bias / 6, projection x 6 in the packing,
  // ops/hip_ops.pack_stem_block0): the stem's and the depthwise's clamps fold into the
  // f32 -> f16 conversion and the last fma (48 of the unrolled loop's ~360 VALU were min / max)
  const f16x4 z4 = {0, 0, 0, 0}, s4 = {1, 1, 1, 1};
  const f16x8 h0 = {0, 0, 0, 0, 0, 0, 0, 0}, h6 = {1, 1, 1, 1, 1, 1, 1, 1};
  f16x8 D[3];
#pragma unroll
  for (int s_ = 0; s_ < 3; ++s_) D[s_] = bdv;
  __syncthreads();  // prologue rows visible

  for (int t0 = 0; t0 < n_st; t0 += U) {
#pragma unroll
    for (int ph = 0; ph < U; ++ph) {
      const int t = t0 + ph;
      const int s = y0 - 1 + t;  // stem row (global)
      // ---- [gather] the next step's rows (pair t + 1) -> IN; its registers refill
      // with pair t + 1 + PD
      {
        const int sl = (ph + 1) % PD;
#pragma unroll
        for (int u = 0; u < GPX; ++u) store_px(2 * (t + 1) + 1 + gk[u], u, xr[sl][u], sto[ph][u]);
#pragma unroll
        for (int u = 0; u < GPX; ++u) xr[sl][u] = fetch_px(2 * (t + 1 + PD) + 1 + gk[u], u);
      }
      // ---- [stem] row s from ring rows 2t .. 2t + 2 -> S[t & 1] (fp16, relu6; 0 outside)
      char* S = S2 + (t & 1) * s_bytes;
      const bool srow = s >= 0 && s < a.SH && t < n_st;  // uniform
      {
        s16x4 xf[3];
#pragma unroll
        for (int m = 0; m < 3; ++m)
          xf[m] = *reinterpret_cast<const s16x4*>(IN + sro[ph][m]);
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          f32x4 e4 = bst[sub];
#pragma unroll
          for (int m = 0; m < 3; ++m) e4 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wst[sub][m], xf[m], e4, 0, 0, 0);
          f16x4 o = {(f16)e4[0], (f16)e4[1], (f16)e4[2], (f16)e4[3]};
          o = __builtin_elementwise_min(__builtin_elementwise_max(o, z4), s4);
          if (!(srow && sin_x)) o = z4;  // depthwise zero padding outside the stem image
          if (sj < NSC) *reinterpret_cast<f16x4*>(S + (size_t)sj * kSP + (sub * 16 + kq * 4) * 2) = o;
        }
      }
      lds_barrier();  // A: stem row complete
      // ---- [depthwise] stem row s feeds output rows s + 1 (ky 0), s (ky 1), s - 1 (ky 2, completes)
      // slots: output o lives in slot (o - y0 + 1) % 3 (static in the unrolled round)
      {
        f16x8 v[3];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) v[kx] = *reinterpret_cast<const f16x8*>(S + (size_t)(xc + kx) * kSP + kq * 16);
        const int s0 = (ph + 1) % 3, s1 = ph % 3, s2 = (ph + 2) % 3;  // o = s+1, s, s-1
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) D[s0] = v[kx] * wdv[kx] + D[s0];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) D[s1] = v[kx] * wdv[3 + kx] + D[s1];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) D[s2] = v[kx] * wdv[6 + kx] + D[s2];
        const int o = s - 1;
        if (o >= y0 && o < y1) {  // uniform
          f16x8 d = __builtin_elementwise_min(__builtin_elementwise_max(D[s2], h0), h6);
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, d, acc, 0, 0, 0);
          if (xv) {
            bf16* orow = a.out + ((size_t)b * a.SH + o) * a.SW * 16;  // uniform
            bf16* op = reinterpret_cast<bf16*>(reinterpret_cast<char*>(orow) + (unsigned)(((x0 + xl) * 16 + kq * 4) * 2));
            const bf16x4 ob = {(bf16)(acc[0] + bpv[0]), (bf16)(acc[1] + bpv[1]), (bf16)(acc[2] + bpv[2]),
                               (bf16)(acc[3] + bpv[3])};
            *reinterpret_cast<bf16x4*>(op) = ob;
          }
        }
        D[s2] = bdv;  // slot reopens as output s + 2 (bias first, as stem_block0_kernel)
      }
      if (!ONEB) lds_barrier();  // two-barrier form (round 4): B, S and IN rows free / visible
    }
  }
}

template <int NW, int GPX, bool ONEB>
void launch_stem_band(const StemBandArgs& a, size_t lds, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_band_kernel<NW, GPX, ONEB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "stem_band attr");
    attr = true;
  }
  hipLaunchKernelGGL((stem_band_kernel<NW, GPX, ONEB>), dim3(a.B * a.nby * a.nbx), dim3(64 * NW), lds, st, a);
  check_launch("stem_band");
}

}  // namespace

size_t stem_band_lds(int SW, int nbx, int R) {
  const int TW = cdiv(SW, nbx);
  const int NSC = TW + 2, NIC = 2 * NSC + 1;
  return (size_t)6 * NIC * 8 + (size_t)2 * NSC * kSP + (size_t)(2 * (R + 2) + 1) * 4;
}

void stem_band(const StemBlock0Params& p, int nbx, hipStream_t st, bool one_barrier) {
  if (p.Cout != 16) throw std::invalid_argument("stem_band: block 0 must project to 16 channels");
  if (p.SH != (p.H - 1) / 2 + 1 || p.SW != (p.W - 1) / 2 + 1) throw std::invalid_argument("stem_band: bad stem size");
  if (nbx < 1 || p.TY < 1) throw std::invalid_argument("stem_band: bad bands");
  const int TW = cdiv(p.SW, nbx);
  const int NW = cdiv(TW + 2, 16);
  const int NIC = 2 * (TW + 2) + 1;
  const int GPX = cdiv(2 * NIC, 64 * NW);
  const size_t lds = stem_band_lds(p.SW, nbx, p.TY);
  if (lds > 160 * 1024) throw std::invalid_argument("stem_band: LDS over 160 KiB");
  StemBandArgs a{p.frames, p.lut_x, p.lut_y, p.ws, p.bs, reinterpret_cast<const f16*>(p.wd),
                 reinterpret_cast<const f16*>(p.bd), reinterpret_cast<const f16*>(p.wp), p.bp, p.out,
                 p.B, p.Hc, p.Wc, p.H, p.W, p.SH, p.SW, p.TY, nbx, cdiv(p.SH, p.TY), TW};
#define SB(NW_, G_)                                                   \
  if (NW == NW_ && GPX == G_) {                                       \
    if (one_barrier) launch_stem_band<NW_, G_, true>(a, lds, st);     \
    else launch_stem_band<NW_, G_, false>(a, lds, st);                \
    return;                                                           \
  }
  // 2 x NIC = 4 (TW + 2) + 2 <= 64 NW + 2: at most 2 gathered pixels per lane
  SB(1, 1) SB(2, 1) SB(3, 1) SB(4, 1) SB(5, 1) SB(6, 1) SB(7, 1) SB(8, 1)
  SB(1, 2) SB(2, 2) SB(3, 2) SB(4, 2) SB(5, 2) SB(6, 2) SB(7, 2) SB(8, 2)
#undef SB
  throw std::invalid_argument("stem_band: no instantiation for this band width");
}

}  // namespace ssa
