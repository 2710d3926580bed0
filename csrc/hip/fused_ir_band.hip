// Row-streaming fused MobileNetV2 inverted residual for the high-resolution blocks
// (blocks 1-6 of DeepLabv3-MobileNetV2 at 513^2: 257^2 -> 129^2 -> 65^2 -> 33^2 maps,
// Cin 16..32, hidden 96..192, Cout 24..64, stride 1 or 2, dilation 1), gfx950.
//
//   out = project( relu6( dw3x3_s( relu6( expand(x) ) ) ) ) [+ x]
//
// Round 1 ran these blocks as 2-D tile kernels (fused_ir / fused_ir_persist): every
// tile re-expanded its input halo (1.3-4.6x the outputs at these tile sizes), and each
// 32-channel hidden chunk cost two workgroup barriers around a few MFMAs, so blocks 1-6
// took 365 us per 32-frame step against a ~40 us HBM/MFMA roofline
// (profiles/r2_v1_layer_times.txt). The reference runs the whole network as one Edge
// TPU call (/root/reference/sem_seg_server.py:162).
//
// Here a workgroup owns a BAND: R output rows x TW = 16 * NW output columns of one
// image, and streams the band's input rows top to bottom:
//   * every input row is expanded exactly once (no vertical halo recompute inside the
//     band; the horizontal halo is 2 columns): MFMA 16x16x32 bf16, A = the block's
//     expansion weights (fragment-packed, LDS), B = 16 input pixels straight from HBM
//     (one 16-byte load per lane, prefetched one row ahead) -> relu6 -> fp16 row E in
//     LDS holding ALL hidden channels of the row;
//   * the depthwise is accumulated per input row into register-resident fp16 partial
//     sums of the 2 (stride 2) or 3 (stride 1) output rows that row feeds: each E read
//     (one 16-byte ds_read per tap column) serves every open output row, so an input
//     pixel is read 3x (not 9x) from LDS;
//   * when an output row's last input row has been added, its depthwise result feeds
//     the projection MFMA (fp16, K = 32 per hidden chunk) as the B fragment directly
//     (lane = 8 channels of one pixel), and the row is stored (+ bias, + residual);
//   * one barrier per input row (two with a single E slot, chosen when two slots
//     would keep the CU below two workgroups).
// Lane -> pixel mapping: wave w owns output columns 16w..16w+15 of the band (MFMA B
// columns), so the depthwise of a lane is the one pixel whose projection it feeds.
// E layout: pixel-major rows of hidP fp16 + 16 B pad (pitch/16 odd: the 16 lanes of a
// ds_read_b128 quarter on consecutive pixels hit distinct 16-byte bank groups); stride-2
// rows are stored even columns first, then odd columns (the even half padded to 8 mod 16
// entries), so the three taps of 16 consecutive outputs read 16 consecutive entries.
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

typedef _Float16 f16;
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// A band spans the FULL map width: NW = ceil(OW / 16) waves, wave w owning output
// columns 16w..16w+15 (9 waves at 129 columns, 5 at 65, 3 at 33). Round-2's first
// version cut 62/63-column bands, and the odd map widths (2^k + 1) left a last band of
// 1-5 columns running a whole workgroup. The band's input row ((OW - 1) * S + 3 pixels)
// then fills ceil(IWT / 16) MFMA pixel groups, S per wave at most.
__host__ __device__ constexpr int band_waves(int OW) { return (OW + 15) / 16; }

struct BandArgs {
  const bf16* in; const char* blob; bf16* out;
  int B, IH, IW, Cin, OH, OW, Cout, residual;
  int R, nbx, nby;          // rows per band, bands across / down
  int TW;                   // output columns per band (<= 16 * NW; < 16 * NW - 1 when split)
  int HE, P, EROW;          // stride-2 even-half entries, E pixel pitch (B), E row bytes
  int blob_bytes;           // host-packed weights, copied to LDS once
  int o_be, o_wd, o_bd, o_wp, o_bp;  // section offsets inside the blob (bytes)
};

// Workgroup barrier for LDS hand-offs only. __syncthreads() is a workgroup release
// fence: with the previous row's output stores pending it makes the compiler drain
// vmcnt to 0 -- which, on the in-order vector memory counter, also waits for the input
// rows prefetched behind those stores and exposed a full HBM round trip per input row.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Host-packed blob: [We frags NSH KiB][be hidP f32][wd 9 x hidP f16][bd hidP f16]
// [Wp frags NS*NCH KiB][bp NS*16 f32]; sections 16-byte aligned. The host folds the
// relu6 scale: expansion weights and bias and the depthwise bias come divided by 6, the
// projection weights multiplied by 6, so both relu6 become [0, 1] clamps that fold into
// the clamp bit of the instruction producing the value (E' = E / 6, D' = D / 6).
// HS = 2 (round 3): two waves per 16-column group, each owning half of the hidden
// channels (expansion sub-tiles, depthwise chunks and the projection's K), twice the waves
// per CU at the same LDS -- the band kernels ran 3-9 waves per CU and were latency-bound
// (block 2: 62 % of wave cycles in s_waitcnt / barrier waits, profiles/r3_band2_pmc.txt).
// The second half's projection partial sums reach the first half through a double-buffered
// LDS exchange behind the next input row's barrier, and the first half stores that output
// row one step later.
template <int S, int NSH, int NS, int NSLOT, int NW, int HS>
__global__ __launch_bounds__(64 * NW * HS) void fused_ir_band_kernel(BandArgs a) {
  constexpr int kBW = NW, kBT = 64 * NW * HS;
  constexpr int NCH = NSH / 2;            // 32-channel hidden chunks
  constexpr int NSHH = (NSH + HS - 1) / HS, NCHH = (NCH + HS - 1) / HS;  // per hidden half
  constexpr int HID = NSH * 16;
  constexpr int NDS = S == 1 ? 3 : 2;     // open output rows (D accumulator slots)
  constexpr int U = S == 1 ? 3 : 4;       // step unroll: static slot roles
  constexpr int GI = S;                   // input pixel groups per wave per row
  constexpr int kTW = 16 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wid = wid_all % NW, hh = wid_all / NW;  // column wave, hidden half
  const int r16 = lane & 15, kq = lane >> 4;

  int blk = blockIdx.x;
  const int bx = blk % a.nbx;
  blk /= a.nbx;
  const int by = blk % a.nby;
  const int b = blk / a.nby;
  const int x0 = bx * a.TW, y0 = by * a.R, y1 = min(y0 + a.R, a.OH);
  const int twv = min(a.TW, a.OW - x0);           // valid output columns of this band
  const int iwv = (twv - 1) * S + 3;              // local input columns it reads
  const int ixb = x0 * S - 1;                     // global column of local input column 0

  // ---- weights -> LDS (16-byte copies)
  for (int i = tid; i < a.blob_bytes / 16; i += kBT)
    *reinterpret_cast<i32x4*>(smem + i * 16) = *reinterpret_cast<const i32x4*>(a.blob + i * 16);
  const char* sWe = smem;
  const float* sBe = reinterpret_cast<const float*>(smem + a.o_be);
  const char* sWd = smem + a.o_wd;
  const char* sBd = smem + a.o_bd;
  const char* sWp = smem + a.o_wp;
  const float* sBp = reinterpret_cast<const float*>(smem + a.o_bp);
  char* sE = smem + ((a.blob_bytes + 15) & ~15);
  // HS = 2: projection partial-sum exchange [2 buffers][NW column waves][NS][64 lanes] f32x4
  f32x4* sX = reinterpret_cast<f32x4*>(sE + NSLOT * a.EROW);
  __syncthreads();  // (the only full barrier: no global store is pending yet)

  // ---- this lane's output pixel and its three tap columns in E
  const int xl = wid * 16 + r16;
  const bool xv = xl < twv;
  const int xc = xv ? xl : 0;
  int ecol[3];
  if (S == 1) {
    ecol[0] = xc * a.P; ecol[1] = (xc + 1) * a.P; ecol[2] = (xc + 2) * a.P;
  } else {
    ecol[0] = xc * a.P; ecol[1] = (a.HE + xc) * a.P; ecol[2] = (xc + 1) * a.P;
  }
  // ---- this wave's input pixel groups: local column i = (wid + k*NW)*16 + r16
  int epix[GI], gcol[GI];
  bool pin[GI];
#pragma unroll
  for (int k = 0; k < GI; ++k) {
    const int g = wid + k * kBW;
    const int i = g * 16 + r16;
    const int ic = i < iwv ? i : 0;
    // columns past the band's input (and out-of-image ones) write into the sink entry
    // at the row's end (an aliased real entry would race with the lane that owns it)
    gcol[k] = ixb + ic;
    pin[k] = i < iwv && gcol[k] >= 0 && gcol[k] < a.IW;
    // out-of-image columns keep the zeros written below (the expansion of a padding
    // pixel goes to the sink instead of being masked per MFMA)
    epix[k] = pin[k] ? (S == 1 ? ic : ((ic & 1) ? a.HE + (ic >> 1) : (ic >> 1))) * a.P : a.EROW - a.P;
  }
  // zero the E entries of this band's out-of-image columns (at most the first and the
  // last local column) in every slot, once: they are never written again
  for (int z = tid; z < NSLOT * 2 * (HID / 8); z += kBT) {
    const int slot = z / (2 * (HID / 8)), rem = z % (2 * (HID / 8));
    const int side = rem / (HID / 8), c8 = rem % (HID / 8);
    const int i = side == 0 ? 0 : iwv - 1;
    const int gc = ixb + i;
    if (gc < 0 || gc >= a.IW) {
      const int e = S == 1 ? i : ((i & 1) ? a.HE + (i >> 1) : (i >> 1));
      *reinterpret_cast<i32x4*>(sE + slot * a.EROW + e * a.P + c8 * 16) = i32x4{0, 0, 0, 0};
    }
  }
  __syncthreads();
  // X fragment loads (B operand): lane = pixel r16, channels kq*8..+7 (zero past Cin)
  const bool kin = kq * 8 < a.Cin;
  // input rows prefetched U steps ahead (slot = step % U, static after the unroll): one
  // step of compute is ~1k cycles against ~2-4k of HBM latency
  bf16x8 xq[U][GI];
  // Branch- and select-free: every lane issues all GI loads, clamped to a valid pixel
  // (a conditional load, or a zero-select right after the load, made the compiler wait
  // for the row just prefetched). No masking is needed: channel-padding lanes read real
  // (finite) channels that meet zero expansion weights, and out-of-image columns are
  // zeroed when E is written; out-of-image rows are never expanded.
  // per-lane element offsets inside a row (fixed for the kernel) against a uniform row base:
  // SGPR base + 32-bit VGPR offset per access instead of 64-bit VALU address arithmetic
  unsigned xoff[GI];
#pragma unroll
  for (int k = 0; k < GI; ++k) xoff[k] = (min(max(gcol[k], 0), a.IW - 1) * a.Cin + (kin ? kq * 8 : 0)) * 2u;  // bytes
  auto load_x = [&](int iy, bf16x8* dst) {
    const int iyc = min(max(iy, 0), a.IH - 1);
    const bf16* row = a.in + ((size_t)b * a.IH + iyc) * a.IW * a.Cin;
#pragma unroll
    for (int k = 0; k < GI; ++k) dst[k] = ld8_at(row, xoff[k]);
  };

  f16x8 D[NDS][NCHH];
#pragma unroll
  for (int s = 0; s < NDS; ++s)
#pragma unroll
    for (int c = 0; c < NCHH; ++c) D[s][c] = f16x8{0, 0, 0, 0, 0, 0, 0, 0};
  // HS = 2, first half: the output row completed last step, waiting for the second half's
  // partial sums (stored after this step's barrier)
  f32x4 pend[NS];
  int pend_o = -1, pend_buf = 0;
  auto store_row = [&](int o, const f32x4 (&acc)[NS]) {
    if (!xv) return;
    const size_t orow = ((size_t)b * a.OH + o) * a.OW;  // uniform
    const int px = x0 + xl;
    const bf16* rrow = a.in + orow * a.Cin;
    bf16* wrow = a.out + orow * a.Cout;
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const int ch = n * 16 + kq * 4;
      if (ch >= a.Cout) continue;
      f32x4 v = acc[n];
      if (a.residual) {  // stride 1, Cin == Cout: same pixel of the input
        const bf16x4 r = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const char*>(rrow) + (unsigned)(px * a.Cin + ch) * 2u);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += (float)r[q];
      }
      const bf16x4 ob = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      *reinterpret_cast<bf16x4*>(reinterpret_cast<char*>(wrow) + (unsigned)(px * a.Cout + ch) * 2u) = ob;
    }
  };
  auto flush_pending = [&]() {  // first half, behind a barrier after the exchange write
    if (HS == 2 && hh == 0 && pend_o >= 0) {
      const f32x4* xs = sX + ((size_t)(pend_buf * NW + wid) * NS) * 64 + lane;
#pragma unroll
      for (int n = 0; n < NS; ++n) pend[n] += xs[n * 64];
      store_row(pend_o, pend);
      pend_o = -1;
    }
  };
  const f16x8 h0 = {0, 0, 0, 0, 0, 0, 0, 0}, h1 = {1, 1, 1, 1, 1, 1, 1, 1};

  const int iy0 = y0 * S - 1;
  const int n_in = (y1 - y0 - 1) * S + 3;
#pragma unroll
  for (int q = 0; q < U; ++q) load_x(iy0 + q, xq[q]);

  // whole unrolled rounds: steps past n_in expand rows nobody reads and feed output
  // rows past the band (skipped), which keeps the round straight-line code (an early
  // exit inside it made the compiler's wait counts at the loop header fall back to 0)
  for (int t0 = 0; t0 < n_in; t0 += U) {
#pragma unroll
    for (int ph = 0; ph < U; ++ph) {
      const int t = t0 + ph;
      const int iy = iy0 + t;
      const bool rowin = iy >= 0 && iy < a.IH;  // uniform
      char* E = sE + (NSLOT == 2 ? (t & 1) : 0) * a.EROW;
      if (NSLOT == 1) lds_barrier();  // every read of the previous row is done
      // ---- [expand] input row iy -> E (fp16, relu6; zero at image columns outside)
      if (rowin) {
#pragma unroll
        for (int hs2 = 0; hs2 < NSHH; ++hs2) {
          const int hs = hh * NSHH + hs2;
          if (HS > 1 && hs >= NSH) break;  // uniform
          const bf16x8 wf = *reinterpret_cast<const bf16x8*>(sWe + hs * 1024 + lane * 16);
          const f32x4 be4 = *reinterpret_cast<const f32x4*>(sBe + hs * 16 + kq * 4);
#pragma unroll
          for (int k = 0; k < GI; ++k) {
            const f32x4 e = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xq[ph][k], be4, 0, 0, 0);
            // relu6 is a [0, 1] clamp on the 1/6-scaled values: the clamp bit of the
            // conversion, no separate max / min
            f16x4 o = {(f16)e[0], (f16)e[1], (f16)e[2], (f16)e[3]};
            o = __builtin_elementwise_min(__builtin_elementwise_max(o, h0.lo), h1.lo);
            *reinterpret_cast<f16x4*>(E + epix[k] + (hs * 16 + kq * 4) * 2) = o;
          }
        }
      }
      // the input pixels of row t + U: in flight under the next U steps
      load_x(iy + U, xq[ph]);  // (past the band's last row: a harmless clamped reload)
      lds_barrier();
      flush_pending();  // the second half's partial sums of last step's row are visible
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
      if (rowin && xv) {
#pragma unroll
        for (int cc = 0; cc < NCHH; ++cc) {
          const int c = hh * NCHH + cc;
          if (HS > 1 && c >= NCH) break;  // uniform
          const int co = (c * 32 + kq * 8) * 2;
          f16x8 v[3];
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) v[kx] = *reinterpret_cast<const f16x8*>(E + ecol[kx] + co);
#pragma unroll
          for (int j = 0; j < nct; ++j) {
            if (orow[j] < y0 || orow[j] >= y1) continue;  // uniform
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const f16x8 w = *reinterpret_cast<const f16x8*>(sWd + ((ky[j] * 3 + kx) * HID) * 2 + co);
              D[sl[j]][cc] = v[kx] * w + D[sl[j]][cc];
            }
          }
        }
      }
      // ---- [complete] the output row whose last input row this was
      const int jc = S == 1 ? 2 : ((ph & 1) ? -1 : 1);
      if (jc >= 0) {
        const int o = orow[jc < 0 ? 0 : jc];
        const int sc = sl[jc < 0 ? 0 : jc];
        if (o >= y0 && o < y1) {
          f32x4 acc[NS];
#pragma unroll
          for (int n = 0; n < NS; ++n)
            acc[n] = hh == 0 ? *reinterpret_cast<const f32x4*>(sBp + n * 16 + kq * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int cc = 0; cc < NCHH; ++cc) {
            const int c = hh * NCHH + cc;
            if (HS > 1 && c >= NCH) break;  // uniform
            const f16x8 bd = *reinterpret_cast<const f16x8*>(sBd + (c * 32 + kq * 8) * 2);
            f16x8 d = D[sc][cc] + bd;
            d = __builtin_elementwise_min(__builtin_elementwise_max(d, h0), h1);
            D[sc][cc] = h0;
#pragma unroll
            for (int n = 0; n < NS; ++n) {
              const f16x8 wp = *reinterpret_cast<const f16x8*>(sWp + (n * NCH + c) * 1024 + lane * 16);
              acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wp, d, acc[n], 0, 0, 0);
            }
          }
          if (HS == 1) {
            store_row(o, acc);
          } else if (hh == 1) {  // partial sums -> exchange buffer (t & 1)
            f32x4* xs = sX + ((size_t)((t & 1) * NW + wid) * NS) * 64 + lane;
#pragma unroll
            for (int n = 0; n < NS; ++n) xs[n * 64] = acc[n];
          } else {
#pragma unroll
            for (int n = 0; n < NS; ++n) pend[n] = acc[n];
            pend_o = o;
            pend_buf = t & 1;
          }
        }
      }
    }
  }
  if (HS == 2) {
    lds_barrier();
    flush_pending();
  }
}

template <int S, int NSH, int NS, int NSLOT, int NW, int HS>
void launch_band(const BandArgs& a, size_t lds, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_ir_band_kernel<S, NSH, NS, NSLOT, NW, HS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "fused_ir_band attr");
    attr = true;
  }
  hipLaunchKernelGGL((fused_ir_band_kernel<S, NSH, NS, NSLOT, NW, HS>), dim3(a.B * a.nby * a.nbx), dim3(64 * NW * HS), lds,
                     st, a);
  check_launch("fused_ir_band");
}

struct BandGeom {
  int IWT, HE, NE, P, EROW;
};

BandGeom band_geom(int stride, int hidP, int OW) {
  BandGeom g;
  const int tw = OW;
  g.IWT = (tw - 1) * stride + 3;
  g.P = hidP * 2 + 16;
  if (stride == 1) {
    g.HE = 0;
    g.NE = g.IWT;
  } else {
    const int even = (g.IWT + 1) / 2;
    g.HE = even + ((8 - even % 16) + 16) % 16;  // == 8 (mod 16)
    g.NE = g.HE + g.IWT / 2;
  }
  g.EROW = (g.NE + 1) * g.P;  // + a sink entry for the padding lanes of the last group
  return g;
}

}  // namespace

// split = 2: the map width is cut into two column bands (129 -> 78 + 51: 5 column waves
// instead of 9, so hs = 2 fits the 1024-thread workgroup); E rows then hold the band's input
// columns only. A band of TW outputs reads (TW - 1) * S + 3 input columns, which the NW * S
// pixel groups of its waves must cover: TW <= 16 * NW - 2.
static int band_tw(int OW, int split) {
  return split == 2 ? 16 * band_waves((OW + 1) / 2) - 2 : OW;
}

size_t fused_ir_band_lds(int stride, int hidP, int OW, int blob_bytes, int nslot, int hs, int Cout, int split) {
  const int tw = band_tw(OW, split);
  const BandGeom g = band_geom(stride, hidP, tw < OW ? tw : OW);
  const size_t xch = hs == 2 ? (size_t)2 * band_waves(split == 2 ? (OW + 1) / 2 : OW) * ((Cout + 15) / 16) * 1024 : 0;
  return (size_t)((blob_bytes + 15) & ~15) + (size_t)nslot * g.EROW + xch;
}

int fused_ir_band_cols(int stride) { (void)stride; return 0; }  // full map width

void fused_ir_band(const FusedBandParams& p, hipStream_t st) {
  if (p.stride != 1 && p.stride != 2) throw std::invalid_argument("fused_ir_band: stride 1 or 2");
  if (p.Cin > 32 || p.Cin % 8 || p.hidP % 32 || p.R < 1) throw std::invalid_argument("fused_ir_band: Cin <= 32, hidP % 32");
  if (p.residual && (p.stride != 1 || p.Cin != p.Cout)) throw std::invalid_argument("fused_ir_band: bad residual");
  if (p.OH != (p.IH - 1) / p.stride + 1 || p.OW != (p.IW - 1) / p.stride + 1)
    throw std::invalid_argument("fused_ir_band: output size must be the pad-1 3x3 conv's");
  const int split = p.split == 2 ? 2 : 1;
  const int tw = band_tw(p.OW, split) < p.OW ? band_tw(p.OW, split) : p.OW;  // band output columns
  const BandGeom g = band_geom(p.stride, p.hidP, tw);
  const int hs = p.hs == 2 ? 2 : 1;
  const size_t lds = fused_ir_band_lds(p.stride, p.hidP, p.OW, p.blob_bytes, p.nslot, hs, p.Cout, split);
  if (lds > 160 * 1024) throw std::invalid_argument("fused_ir_band: LDS over 160 KiB");
  BandArgs a{p.in, reinterpret_cast<const char*>(p.blob), p.out, p.B, p.IH, p.IW, p.Cin, p.OH, p.OW, p.Cout,
             p.residual, p.R, cdiv(p.OW, tw), cdiv(p.OH, p.R), tw, g.HE, g.P, g.EROW, p.blob_bytes,
             p.o_be, p.o_wd, p.o_bd, p.o_wp, p.o_bp};
  const int NSH = p.hidP / 16, NS = (p.Cout + 15) / 16;
  const int NW = band_waves(split == 2 ? (p.OW + 1) / 2 : p.OW);
  if ((tw - 1) * p.stride + 3 > 16 * NW * p.stride) throw std::invalid_argument("fused_ir_band: band too wide");
#define BAND(S_, NSH_, NS_, NW_)                                                 \
  if (p.stride == S_ && NSH == NSH_ && NS == NS_ && NW == NW_) {                 \
    if (hs == 2) {  /* 2 x NW waves must fit 1024 threads: NW <= 8 */            \
      if (NW_ > 8) throw std::invalid_argument("fused_ir_band: hs 2 needs <= 8 column waves"); \
      if (p.nslot == 2) launch_band<S_, NSH_, NS_, 2, NW_, (NW_ > 8 ? 1 : 2)>(a, lds, st); \
      else launch_band<S_, NSH_, NS_, 1, NW_, (NW_ > 8 ? 1 : 2)>(a, lds, st);    \
    } else if (p.nslot == 2) launch_band<S_, NSH_, NS_, 2, NW_, 1>(a, lds, st);  \
    else launch_band<S_, NSH_, NS_, 1, NW_, 1>(a, lds, st);                      \
    return;                                                                      \
  }
  // block 1 (16 -> 96 -> 24, s2), 2 (24 -> 144 -> 24), 3 (24 -> 144 -> 32, s2),
  // 4-5 (32 -> 192 -> 32), 6 (32 -> 192 -> 64, s2); hidden 144 runs padded to 160
  // (map widths at 513^2: 129, 129, 65, 65, 33)
  BAND(2, 6, 2, 9) BAND(1, 10, 2, 9) BAND(2, 10, 2, 5) BAND(1, 12, 2, 5) BAND(2, 12, 4, 3)
  // blocks 1-2 in two column bands (split = 2: 5 column waves)
  BAND(2, 6, 2, 5) BAND(1, 10, 2, 5)
#undef BAND
  throw std::invalid_argument("fused_ir_band: no instantiation for this (stride, hidden, Cout)");
}

}  // namespace ssa
