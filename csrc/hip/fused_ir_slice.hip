// Hidden-sliced row-streaming fused MobileNetV2 inverted residual (blocks 1-6 of
// DeepLabv3-MobileNetV2 at 513^2: Cin 16..32, hidden 96..192, Cout 24..64, stride 1 or 2),
// gfx950.
//
//   out = project( relu6( dw3x3_s( relu6( expand(x) ) ) ) ) [+ x]
//
// Same row streaming as fused_ir_band.hip (a workgroup owns R output rows x TW columns of
// one image, every input row is expanded once into an on-chip fp16 row E, the depthwise
// accumulates per input row in registers), but the waves split the HIDDEN channels
// instead of each wave doing all of them:
//
//   wave (g, c) = column group g (16 output columns) x hidden chunk c (32 channels).
//
// Why: in the band kernel every wave walks all hidden chunks and re-reads the chunk's
// expansion / depthwise / projection weights from LDS on every input row. Counted per
// input row and wave for block 2 (hidden 160): ~80 of ~105 LDS instructions were weight
// reads, and the LDS pipe -- not the VALU, MFMA or HBM -- set the pace (PMC: 1882 LDS
// instructions and 9371 LDS cycles per wave, 62 % of wave cycles waiting;
// profiles/r3_band2_pmc.txt). Here a wave's weights are ONE chunk's and stay in VGPRs for
// the whole kernel (expansion A fragments, expansion bias, 9 depthwise taps, depthwise
// bias: ~56 VGPRs); per input row a wave issues 2-4 E writes and 3 E reads. The
// projection needs all chunks: the finished depthwise row goes to LDS as exactly the
// projection MFMA's B fragments ([g][c][64 lanes][16 B]), and wave (g, n) for n < NS
// reduces K over the chunks with the fp16 projection fragments (LDS) into output channels
// n*16..n*16+15, + bias (+ residual), bf16 store.
//
// Per input row (one step), two workgroup barriers:
//   [expand row t -> E] [projection of the row completed at step t-1]  | A |
//   [depthwise of row t -> open output rows; completed row -> D-buffer] | B |
// E and the D-buffer are single-buffered: each is written and read on opposite sides of
// a barrier. ONEB (round 5): E and the D-buffer double-buffered by step parity and the
// projection of a completed row deferred by two steps, so ONE barrier per input row is
// enough (E[t&1]: written before barrier t, read after it, rewritten before barrier t+2;
// D[t&1]: written after barrier t, projected before barrier t+2, rewritten after it). Weight blob: pack_fused_band's (relu6 scale folded: both clamps are [0, 1]).
// Reference parity: the model executed is the reference's Edge TPU DeepLabv3-MobileNetV2
// (/root/reference/sem_seg_server.py:238,162).
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

typedef _Float16 f16;
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct SliceArgs {
  const bf16* in; const char* blob; bf16* out;
  int B, IH, IW, Cin, OH, OW, Cout, residual;
  int R, nbx, nby, TW;      // rows per band, bands across / down, output columns per band
  int HE, P, EROW;          // stride-2 even-half entries, E pixel pitch (B), E row bytes
  int hidP, o_be, o_wd, o_bd, o_wp, o_bp;
};

__device__ __forceinline__ void lds_barrier() {
  // LDS hand-offs only: a full __syncthreads() would also drain vmcnt, i.e. wait for the
  // input rows prefetched behind the previous row's output stores
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// S: stride; NCH: hidden chunks of 32; NS: output subtiles of 16; NW: column groups;
// PD: input rows prefetched ahead (U = the step unroll that keeps slot roles static)
template <int S, int NCH, int NS, int NW, bool ONEB>
__global__ __launch_bounds__(64 * NW * NCH) void fused_ir_slice_kernel(SliceArgs a) {
  constexpr int NT = 64 * NW * NCH;
  constexpr int NDS = S == 1 ? 3 : 2;     // open output rows
  constexpr int U = S == 1 ? 3 : 4;       // step unroll: static D-slot roles
  constexpr int PD = S == 1 ? 3 : 2;      // prefetch depth (rows); slot = ph % PD
  constexpr int GI = S;                   // input pixel groups per wave per row
  static_assert(NS <= NCH, "projection tasks run on waves (g, n < NS)");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wid % NW, c = wid / NW;   // column group, hidden chunk
  const int r16 = lane & 15, kq = lane >> 4;

  int blk = blockIdx.x;
  const int bx = blk % a.nbx;
  blk /= a.nbx;
  const int by = blk % a.nby;
  const int b = blk / a.nby;
  const int x0 = bx * a.TW, y0 = by * a.R, y1 = min(y0 + a.R, a.OH);
  const int twv = min(a.TW, a.OW - x0);
  const int iwv = (twv - 1) * S + 3;
  const int ixb = x0 * S - 1;

  // ---- LDS: [Wp frags NS*NCH KiB][bp NS*16 f32][E row(s)][D-buffer(s) NW*NCH KiB]
  constexpr int NB = ONEB ? 2 : 1;
  char* sWp = smem;
  float* sBp = reinterpret_cast<float*>(smem + NS * NCH * 1024);
  char* sE0 = smem + NS * NCH * 1024 + NS * 64;
  char* sD0 = sE0 + NB * a.EROW;
  constexpr int DB = NW * NCH * 1024;
  for (int i = tid; i < NS * NCH * 64; i += NT)
    *reinterpret_cast<i32x4*>(sWp + i * 16) = *reinterpret_cast<const i32x4*>(a.blob + a.o_wp + i * 16);
  for (int i = tid; i < NS * 16; i += NT) sBp[i] = reinterpret_cast<const float*>(a.blob + a.o_bp)[i];

  // ---- this wave's chunk weights -> VGPRs (for the whole kernel)
  bf16x8 wf[2];
  f32x4 be4[2];
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
    const int hs = 2 * c + sub;
    wf[sub] = *reinterpret_cast<const bf16x8*>(a.blob + hs * 1024 + lane * 16);
    be4[sub] = *reinterpret_cast<const f32x4*>(a.blob + a.o_be + (hs * 16 + kq * 4) * 4);
  }
  f16x8 wdv[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
    wdv[tap] = *reinterpret_cast<const f16x8*>(a.blob + a.o_wd + (tap * a.hidP + c * 32 + kq * 8) * 2);
  const f16x8 bdv = *reinterpret_cast<const f16x8*>(a.blob + a.o_bd + (c * 32 + kq * 8) * 2);

  // ---- this lane's output column and its three tap entries in E
  const int xl = g * 16 + r16;
  const bool xv = xl < twv;
  const int xc = xv ? xl : 0;
  int ecol[3];
  if (S == 1) {
    ecol[0] = xc * a.P; ecol[1] = (xc + 1) * a.P; ecol[2] = (xc + 2) * a.P;
  } else {
    ecol[0] = xc * a.P; ecol[1] = (a.HE + xc) * a.P; ecol[2] = (xc + 1) * a.P;
  }
  const int cofs = (c * 32 + kq * 8) * 2;  // this lane's channel offset in an E entry (bytes)
  // ---- this wave's input pixel groups: local column i = (g + k*NW)*16 + r16
  int epix[GI], gcol[GI];
#pragma unroll
  for (int k = 0; k < GI; ++k) {
    const int i = (g + k * NW) * 16 + r16;
    const int ic = i < iwv ? i : 0;
    gcol[k] = ixb + ic;
    const bool pin = i < iwv && gcol[k] >= 0 && gcol[k] < a.IW;
    // padding lanes and out-of-image columns write the sink entry at the row's end
    epix[k] = pin ? (S == 1 ? ic : ((ic & 1) ? a.HE + (ic >> 1) : (ic >> 1))) * a.P : a.EROW - a.P;
  }
  // zero this chunk's slice of the band's out-of-image E columns (never written again)
  for (int z = lane; z < 2 * 4; z += 64) {
    const int side = z >> 2, c8 = z & 3;
    const int i = side == 0 ? 0 : iwv - 1;
    const int gc = ixb + i;
    if (g == 0 && (gc < 0 || gc >= a.IW)) {
      const int e = S == 1 ? i : ((i & 1) ? a.HE + (i >> 1) : (i >> 1));
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        *reinterpret_cast<i32x4*>(sE0 + nb * a.EROW + e * a.P + (c * 32 + c8 * 8) * 2) = i32x4{0, 0, 0, 0};
    }
  }
  __syncthreads();  // (the only full barrier: no global store is pending yet)

  const bool kin = kq * 8 < a.Cin;
  // per-lane element offsets inside a row, fixed for the kernel: the row base is uniform
  // (a scalar 64-bit pointer), so every load / store below is SGPR base + 32-bit VGPR
  // offset -- no per-access 64-bit address arithmetic on the VALU (~120 of the unrolled
  // loop's ~410 VALU were address math)
  unsigned xoff[GI];
#pragma unroll
  for (int k = 0; k < GI; ++k) xoff[k] = (min(max(gcol[k], 0), a.IW - 1) * a.Cin + (kin ? kq * 8 : 0)) * 2u;  // bytes
  bf16x8 xq[PD][GI];
  auto load_x = [&](int iy, bf16x8* dst) {
    // clamped, branch-free: padding-channel lanes read real channels that meet zero
    // expansion weights; out-of-image rows are never expanded
    const int iyc = min(max(iy, 0), a.IH - 1);
    const bf16* row = a.in + ((size_t)b * a.IH + iyc) * a.IW * a.Cin;
#pragma unroll
    for (int k = 0; k < GI; ++k) dst[k] = ld8_at(row, xoff[k]);
  };

  f16x8 D[NDS];
#pragma unroll
  for (int s = 0; s < NDS; ++s) D[s] = f16x8{0, 0, 0, 0, 0, 0, 0, 0};
  const f16x8 h0 = {0, 0, 0, 0, 0, 0, 0, 0}, h1 = {1, 1, 1, 1, 1, 1, 1, 1};
  const bool task = c < NS;  // wave (g, n = c) projects output channels n*16..+15
  int pend_o = -1;           // output row waiting in the D-buffer (uniform)
  int pend2[2] = {-1, -1};   // ONEB: output row waiting in D-buffer [parity] (uniform)

  auto project = [&](int o, const char* sD) {  // sD holds output row o's depthwise (all chunks)
    if (!task) return;
    f32x4 acc = *reinterpret_cast<const f32x4*>(sBp + c * 16 + kq * 4);
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {
      const f16x8 wp = *reinterpret_cast<const f16x8*>(sWp + (c * NCH + cc) * 1024 + lane * 16);
      const f16x8 d = *reinterpret_cast<const f16x8*>(sD + ((g * NCH + cc) * 64 + lane) * 16);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wp, d, acc, 0, 0, 0);
    }
    const int ch = c * 16 + kq * 4;
    if (!xv || ch >= a.Cout) return;
    const size_t orow = ((size_t)b * a.OH + o) * a.OW;  // uniform
    const int px = x0 + xl;
    if (a.residual) {  // stride 1, Cin == Cout: the same pixel of the input
      const bf16x4 r = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const char*>(a.in + orow * a.Cin) + (unsigned)(px * a.Cin + ch) * 2u);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += (float)r[q];
    }
    const bf16x4 ob = {(bf16)acc[0], (bf16)acc[1], (bf16)acc[2], (bf16)acc[3]};
    *reinterpret_cast<bf16x4*>(reinterpret_cast<char*>(a.out + orow * a.Cout) + (unsigned)(px * a.Cout + ch) * 2u) = ob;
  };

  const int iy0 = y0 * S - 1;
  const int n_in = (y1 - y0 - 1) * S + 3;
#pragma unroll
  for (int q = 0; q < PD; ++q) load_x(iy0 + q, xq[q]);

  for (int t0 = 0; t0 < n_in; t0 += U) {
#pragma unroll
    for (int ph = 0; ph < U; ++ph) {
      const int t = t0 + ph;
      const int iy = iy0 + t;
      const bool rowin = iy >= 0 && iy < a.IH;  // uniform
      const int slot = ph % PD;
      char* sE = sE0 + (ONEB ? (t & 1) * a.EROW : 0);
      char* sD = sD0 + (ONEB ? (t & 1) * DB : 0);
      // ---- [expand] input row iy -> E (this wave's 32 hidden channels)
      if (rowin) {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int k = 0; k < GI; ++k) {
            const f32x4 e = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[sub], xq[slot][k], be4[sub], 0, 0, 0);
            f16x4 o = {(f16)e[0], (f16)e[1], (f16)e[2], (f16)e[3]};
            o = __builtin_elementwise_min(__builtin_elementwise_max(o, h0.lo), h1.lo);
            *reinterpret_cast<f16x4*>(sE + epix[k] + ((2 * c + sub) * 16 + kq * 4) * 2) = o;
          }
      }
      load_x(iy + PD, xq[slot]);  // in flight under the next PD steps
      // ---- [project] the row the previous step completed (D-buffer read before barrier A);
      // ONEB: the row completed two steps ago, in D-buffer [t & 1]
      if (ONEB) {
        if (pend2[t & 1] >= 0) {
          project(pend2[t & 1], sD);
          pend2[t & 1] = -1;
        }
      } else if (pend_o >= 0) {
        project(pend_o, sD);
        pend_o = -1;
      }
      lds_barrier();  // A: E row complete; D-buffer free
      // ---- [depthwise] row iy into the open output rows it feeds
      // stride 1: output y0+t (ky 0, slot t%3), y0+t-1 (ky 1), y0+t-2 (ky 2, completes)
      // stride 2: t even -> y0+t/2 (ky 0), y0+t/2-1 (ky 2, completes); t odd -> ky 1
      const int nct = S == 1 ? 3 : ((ph & 1) ? 1 : 2);
      int ky[3], sl[3], orow[3];
      if (S == 1) {
        ky[0] = 0; sl[0] = ph % 3;       orow[0] = y0 + t;
        ky[1] = 1; sl[1] = (ph + 2) % 3; orow[1] = y0 + t - 1;
        ky[2] = 2; sl[2] = (ph + 1) % 3; orow[2] = y0 + t - 2;
      } else if ((ph & 1) == 0) {
        ky[0] = 0; sl[0] = (ph / 2) % 2;     orow[0] = y0 + t / 2;
        ky[1] = 2; sl[1] = (ph / 2 + 1) % 2; orow[1] = y0 + t / 2 - 1;
        ky[2] = 0; sl[2] = 0;                orow[2] = -1;
      } else {
        ky[0] = 1; sl[0] = ((ph - 1) / 2) % 2; orow[0] = y0 + (t - 1) / 2;
        ky[1] = 0; sl[1] = 0;                  orow[1] = -1;
        ky[2] = 0; sl[2] = 0;                  orow[2] = -1;
      }
      if (rowin) {
        f16x8 v[3];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) v[kx] = *reinterpret_cast<const f16x8*>(sE + ecol[kx] + cofs);
#pragma unroll
        for (int j = 0; j < nct; ++j) {
          if (orow[j] < y0 || orow[j] >= y1) continue;  // uniform
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) D[sl[j]] = v[kx] * wdv[ky[j] * 3 + kx] + D[sl[j]];
        }
      }
      // ---- [complete] the output row whose last input row this was -> D-buffer
      const int jc = S == 1 ? 2 : ((ph & 1) ? -1 : 1);
      if (jc >= 0) {
        const int o = orow[jc < 0 ? 0 : jc];
        const int sc = sl[jc < 0 ? 0 : jc];
        if (o >= y0 && o < y1) {  // uniform
          f16x8 d = D[sc] + bdv;
          d = __builtin_elementwise_min(__builtin_elementwise_max(d, h0), h1);
          D[sc] = h0;
          *reinterpret_cast<f16x8*>(sD + ((g * NCH + c) * 64 + lane) * 16) = d;
          if (ONEB) pend2[t & 1] = o;
          else pend_o = o;
        }
      }
      if (!ONEB) lds_barrier();  // B: depthwise reads of E done; D-buffer complete
    }
  }
  if (ONEB) {
    lds_barrier();  // the last steps' D-buffer rows complete
    // in completion order: the older row first (steps n_in-2, n_in-1 by parity)
    const int tl = (n_in + U - 1) / U * U;  // steps run (the unrolled loop rounds up)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int par = (tl + k) & 1;
      if (pend2[par] >= 0) project(pend2[par], sD0 + par * DB);
    }
  } else if (pend_o >= 0) {
    project(pend_o, sD0);
  }
}

template <int S, int NCH, int NS, int NW, bool ONEB>
void launch_slice(const SliceArgs& a, size_t lds, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_ir_slice_kernel<S, NCH, NS, NW, ONEB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "fused_ir_slice attr");
    attr = true;
  }
  hipLaunchKernelGGL((fused_ir_slice_kernel<S, NCH, NS, NW, ONEB>), dim3(a.B * a.nby * a.nbx),
                     dim3(64 * NW * NCH), lds, st, a);
  check_launch("fused_ir_slice");
}

struct SliceGeom {
  int TW, nbx, IWT, HE, NE, P, EROW;
};

// the band's output columns: the widest band its NW column groups cover (stride 1: TW + 2
// input columns <= 16 NW; stride 2: 2 TW + 1 <= 32 NW), then equal bands across OW
SliceGeom slice_geom(int stride, int hidP, int OW, int nw) {
  SliceGeom g;
  const int twmax = stride == 1 ? 16 * nw - 2 : 16 * nw - 1;
  g.nbx = cdiv(OW, twmax);
  g.TW = cdiv(OW, g.nbx);
  g.IWT = (g.TW - 1) * stride + 3;
  g.P = hidP * 2 + 16;
  if (stride == 1) {
    g.HE = 0;
    g.NE = g.IWT;
  } else {
    const int even = (g.IWT + 1) / 2;
    g.HE = even + ((8 - even % 16) + 16) % 16;  // == 8 (mod 16): the odd half's taps hit other banks
    g.NE = g.HE + g.IWT / 2;
  }
  g.EROW = (g.NE + 1) * g.P;  // + the sink entry
  return g;
}

}  // namespace

size_t fused_ir_slice_lds(int stride, int hidP, int OW, int Cout, int nw, bool one_barrier) {
  const int NCH = hidP / 32, NS = (Cout + 15) / 16, NB = one_barrier ? 2 : 1;
  const SliceGeom g = slice_geom(stride, hidP, OW, nw);
  return (size_t)NS * NCH * 1024 + NS * 64 + NB * ((size_t)g.EROW + (size_t)nw * NCH * 1024);
}

void fused_ir_slice(const FusedBandParams& p, int nw, hipStream_t st, bool one_barrier) {
  if (p.stride != 1 && p.stride != 2) throw std::invalid_argument("fused_ir_slice: stride 1 or 2");
  if (p.Cin > 32 || p.Cin % 8 || p.hidP % 32 || p.R < 1) throw std::invalid_argument("fused_ir_slice: Cin <= 32, hidP % 32");
  if (p.residual && (p.stride != 1 || p.Cin != p.Cout)) throw std::invalid_argument("fused_ir_slice: bad residual");
  if (p.OH != (p.IH - 1) / p.stride + 1 || p.OW != (p.IW - 1) / p.stride + 1)
    throw std::invalid_argument("fused_ir_slice: output size must be the pad-1 3x3 conv's");
  const SliceGeom g = slice_geom(p.stride, p.hidP, p.OW, nw);
  const size_t lds = fused_ir_slice_lds(p.stride, p.hidP, p.OW, p.Cout, nw, one_barrier);
  if (lds > 160 * 1024) throw std::invalid_argument("fused_ir_slice: LDS over 160 KiB");
  if ((g.TW - 1) * p.stride + 3 > 16 * nw * p.stride) throw std::invalid_argument("fused_ir_slice: band too wide");
  SliceArgs a{p.in, reinterpret_cast<const char*>(p.blob), p.out, p.B, p.IH, p.IW, p.Cin, p.OH, p.OW, p.Cout,
              p.residual, p.R, g.nbx, cdiv(p.OH, p.R), g.TW, g.HE, g.P, g.EROW, p.hidP,
              p.o_be, p.o_wd, p.o_bd, p.o_wp, p.o_bp};
  const int NCH = p.hidP / 32, NS = (p.Cout + 15) / 16;
#define SLICE(S_, NCH_, NS_, NW_)                                                  \
  if (p.stride == S_ && NCH == NCH_ && NS == NS_ && nw == NW_) {                   \
    if (one_barrier) launch_slice<S_, NCH_, NS_, NW_, true>(a, lds, st);           \
    else launch_slice<S_, NCH_, NS_, NW_, false>(a, lds, st);                      \
    return;                                                                        \
  }
  // block 1 (16 -> 96 -> 24, s2), 2 (24 -> 144 -> 24; hidden padded to 160), 3 (24 -> 144 -> 32,
  // s2), 4-5 (32 -> 192 -> 32), 6 (32 -> 192 -> 64, s2); waves = NW x NCH <= 16
  SLICE(2, 3, 2, 5) SLICE(2, 3, 2, 4) SLICE(1, 5, 2, 3) SLICE(1, 5, 2, 2) SLICE(2, 5, 2, 3) SLICE(2, 5, 2, 2)
  SLICE(1, 6, 2, 2) SLICE(2, 6, 4, 2) SLICE(1, 6, 2, 1) SLICE(2, 6, 4, 1)
#undef SLICE
  throw std::invalid_argument("fused_ir_slice: no instantiation for this (stride, hidden, Cout, waves)");
}

}  // namespace ssa
