// Fused MobileNetV2 inverted residual for the output-stride-16 stage (blocks 7-16 of
// DeepLabv3-MobileNetV2 at 513^2: 33x33 maps, stride 1, dilation 1 or 2, hidden
// 384..960 channels, Cout 64..320), gfx950.
//
//   out = project( relu6( dw3x3_dil( relu6( expand(x) ) ) ) ) [+ x]
//
// The 6x-expanded tensor never leaves the CU. Round 1 ran these blocks
// as pw_conv -> fp16 HBM tensor (up to 67 MB per block at B = 32) -> dw_proj_rows,
// ~540 us for the stage; the reference runs the whole network as one Edge TPU call
// (/root/reference/sem_seg_server.py:162).
//
// Work decomposition (MI355X-first):
//   * one 512-thread workgroup (8 waves, 2 per SIMD) per SPAN: a run of ~HW/S
//     consecutive output pixels of one image in raster order (S = 8 spans per 33x33
//     image -> 136/137 pixels, 9 MFMA pixel groups; B = 32 gives exactly 256
//     workgroups = one per CU). A span covers whole rows except at its two ends, so
//     its expansion halo (every in-image pixel within Chebyshev distance `dil`) is
//     ~1.5x (dil 1) / ~2x (dil 2) the outputs, against 1.4x / 1.9x for an 11x11 tile
//     that would also leave 288 tiles on 256 CUs. The halo pixel list of every span is
//     a host-built table (ops/fused_span.py span_table);
//   * the input halo X stays in VGPRs for the whole kernel (MFMA B fragments, one
//     16-byte load per lane per 32-channel K step); a third halo round (dilation 2)
//     sits in LDS so the 160 -> 320 block stays within 256 VGPRs;
//   * hidden channels stream in 32-wide chunks through three stages, SOFTWARE-
//     PIPELINED over the chunks with ONE barrier per step (step t runs all three on
//     different chunks; the first version ran them back to back with two barriers per
//     chunk and was latency-bound: its per-workgroup time did not change when the
//     span was halved, scripts/bench_span.py --trace):
//       [A] expansion  of chunk t:   E[t&1][halo px, 32] = relu6(X We^T + be), bf16 MFMA
//       [B] depthwise  of chunk t-1: D[..][out px, 32] = relu6(dw(E) + bd), packed fp16
//           VALU, written in projection B-fragment order (1 KiB per 16-pixel group)
//       [C] projection of chunk t-2: acc[out px, Cout] += Wp D, fp16 MFMA, fp32
//           accumulators in VGPRs; waves split as NPI pixel-group sets x 8/NPI Cout slices
//     E and D are double-buffered; the host-packed weights (MFMA fragment order, so
//     every fragment read is a lane-linear 1 KiB ds_read_b128) live in three LDS rings
//     read at the lag of their stage: We [2 slots], misc = wd/bd/be [3], Wp [2];
//   * the weights of step t+1 are fetched into VGPRs by waves 1-7 during step t-1..t
//     and committed to LDS before step t's barrier (plain loads survive the barriers;
//     an LDS-DMA would be drained by the compiler at the first LDS read after it);
//   * E is stored as 4 channel-octet planes [octet][row][WCP] x 16 B with the row
//     pitch WCP = W + 16 (== W mod 16) and planes a multiple of 256 B apart: the 16
//     lanes of every ds_read_b128 lane group (consecutive span pixels, one or two
//     octets) hit 16 distinct 16-byte bank slots, across row wraps too -- the
//     depthwise reads are bank-conflict free (round 1's dw_proj_rows had ~1:1
//     conflict cycles per LDS instruction, profiles/r1_hip_v10_pmc_summary.txt).
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

typedef _Float16 f16;
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int kSNW = 8;         // waves per workgroup
constexpr int kSNT = 64 * kSNW;
constexpr int kSOG = 9;         // max output pixel groups per span (144 pixels)
constexpr int kHdr = 4;         // span table header ints: p0, p1, wy0, nh

struct SpanArgs {
  const bf16* in; const char* w; const float* bp; const int* table; bf16* out;
  int B, H, W, Cin, Cout, NC, S, dil, residual, WCP, WR, hstride, xslots;
  long long* trace;  // debug: s_memtime stamps [block][wave 0/1][64], nullptr normally
};

__host__ __device__ inline int span_plane_bytes(int WR, int WCP) { return (WR * WCP + 15) / 16 * 16 * 16; }

// Debug timeline (a.trace != nullptr): lane 0 of waves 0 and 1 stamp s_memtime at
// phase boundaries of the first chunks (vector stores into the trace buffer).
#define SPAN_STAMP(slot)                                                                     \
  do {                                                                                       \
    if (a.trace && wid < 2 && lane == 0 && (slot) < 64)                                      \
      a.trace[((size_t)blockIdx.x * 2 + wid) * 64 + (slot)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

// Make the compiler's wait-count scoreboard retire a value here: an (empty) inline asm
// that reads the registers forces the s_waitcnt for their pending loads at this point.
// Without it, loads the scoreboard cannot prove complete at the chunk loop's header
// (the halo X prologue loads; staging loads consumed on one path only) are waited for
// with vmcnt(0) inside the loop -- which drains the next chunk's in-flight staging
// loads and exposed a full L2 round trip per chunk in the first version.
template <class T>
__device__ __forceinline__ void retire(const T& v) { asm volatile("" ::"v"(v)); }

template <int KS, int NS, int NPI, int XG>
__global__ __launch_bounds__(kSNT) void fused_ir_span_kernel(SpanArgs a) {
  constexpr int NCI = kSNW / NPI;        // Cout slices
  constexpr int NSW = NS / NCI;          // 16-channel Cout subtiles per wave
  constexpr int GPW = (kSOG + NPI - 1) / NPI;
  constexpr int CH = (2 * KS + NS + 1) * 1024;  // global chunk image: We | Wp | misc
  constexpr int WEB = 2 * KS * 1024, WPB = NS * 1024;
  constexpr int NPC = CH / 16;                  // 16-byte pieces per chunk
  constexpr int NSTG = kSNT - 64;               // staging threads (waves 1..7)
  constexpr int NLD = (NPC + NSTG - 1) / NSTG;
  constexpr int XR = XG < 2 ? XG : 2;
  // the 160 -> 320 block sits at ~250 VGPRs: keep its stages from interleaving
  constexpr bool TIGHT = KS * 4 * XR + GPW * NSW * 4 >= 120;
  static_assert(NS % NCI == 0, "Cout subtiles must split evenly over the Cout slices");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int PLANE = span_plane_bytes(a.WR, a.WCP);
  char* sWe = smem;                    // [2][WEB]
  char* sMisc = sWe + 2 * WEB;         // [3][1024]: wd [9][32] f16 | bd [32] f16 | be [32] f32
  char* sWp = sMisc + 3 * 1024;        // [2][WPB]
  char* sE = sWp + 2 * WPB;            // [2][4 * PLANE]
  char* sD = sE + 8 * PLANE;           // [2][kSOG][1024]
  char* sX = sD + 2 * kSOG * 1024;     // third-round halo X [slot][k] x 1 KiB

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int b = blockIdx.x / a.S, j = blockIdx.x - (blockIdx.x / a.S) * a.S;
  const int* tb = a.table + (size_t)j * a.hstride;
  const int p0 = tb[0], p1 = tb[1], wy0 = tb[2], nh = tb[3];
  const int HW = a.H * a.W, d = a.dil, NC = a.NC;
  const int HG = (nh + 15) >> 4;        // halo pixel groups
  const int OGn = (p1 - p0 + 15) >> 4;  // output pixel groups (<= kSOG, host-checked)
  const int pi = wid % NPI, ci = wid / NPI;

  SPAN_STAMP(0);
  // ---- prologue: We[0] + misc[0] -> ring slot 0, E zeroed (padding taps read 0)
  for (int i = tid; i < WEB / 16; i += kSNT)
    *reinterpret_cast<i32x4*>(sWe + i * 16) = *reinterpret_cast<const i32x4*>(a.w + i * 16);
  if (tid < 64)
    *reinterpret_cast<i32x4*>(sMisc + tid * 16) = *reinterpret_cast<const i32x4*>(a.w + WEB + WPB + tid * 16);
  // zero: E (padding taps), D and the Wp ring and misc slot 2 (the pipeline's fill steps
  // run every stage unconditionally: [C] at t < 2 adds 0 * 0, [B] at t = 0 makes zeros)
  for (int i = tid; i < PLANE / 2; i += kSNT) *reinterpret_cast<i32x4*>(sE + i * 16) = i32x4{0, 0, 0, 0};
  for (int i = tid; i < 2 * kSOG * 64; i += kSNT) *reinterpret_cast<i32x4*>(sD + i * 16) = i32x4{0, 0, 0, 0};
  for (int i = tid; i < 2 * WPB / 16; i += kSNT) *reinterpret_cast<i32x4*>(sWp + i * 16) = i32x4{0, 0, 0, 0};
  if (tid < 64) *reinterpret_cast<i32x4*>(sMisc + 2048 + tid * 16) = i32x4{0, 0, 0, 0};

  // staging: piece i of a step's set = We[t+1] (i < WEB/16) | misc[t+1] | Wp[t-1].
  // Branch-free (per-piece branches split the step into basic blocks the scheduler
  // cannot hoist LDS reads across): every piece loads from a valid address (chunk 0
  // when its part is idle this step) and idle pieces are stored to a 16-byte sink.
  const bool stager = wid > 0;
  const int st = tid - 64;
  i32x4 stg[NLD];
  int sprt[NLD], soff[NLD];  // part (0 We, 1 misc, 2 Wp, 3 none) and byte offset in it
#pragma unroll
  for (int q = 0; q < NLD; ++q) {
    stg[q] = i32x4{0, 0, 0, 0};
    const int i = st + q * NSTG;
    sprt[q] = !stager || i >= NPC ? 3 : i < WEB / 16 ? 0 : i < WEB / 16 + 64 ? 1 : 2;
    soff[q] = sprt[q] == 0 ? i * 16 : sprt[q] == 1 ? (i - WEB / 16) * 16 : sprt[q] == 2 ? (i - WEB / 16 - 64) * 16 : 0;
  }
  char* sink = sX + (size_t)a.xslots * KS * 1024;  // 16 bytes past the last region
  auto stage_load = [&](int cw, int cp) {
    const bool okw = cw < NC, okp = cp >= 0 && cp < NC;
    const char* bw = a.w + (size_t)(okw ? cw : 0) * CH;
    const char* bp = a.w + (size_t)(okp ? cp : 0) * CH;
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const char* src = sprt[q] == 0 ? bw + soff[q] : sprt[q] == 1 ? bw + WEB + WPB + soff[q] : bp + WEB + soff[q];
      stg[q] = *reinterpret_cast<const i32x4*>(sprt[q] == 3 ? a.w : src);
    }
  };
  auto stage_store = [&](int cw, int cp) {
    const bool okw = cw < NC, okp = cp >= 0 && cp < NC;
    char* dw = sWe + (cw & 1) * WEB;
    char* dm = sMisc + (cw % 3) * 1024;
    char* dp = sWp + (cp & 1) * WPB;
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      char* dst = sprt[q] == 0 ? (okw ? dw + soff[q] : sink)
                : sprt[q] == 1 ? (okw ? dm + soff[q] : sink)
                : sprt[q] == 2 ? (okp ? dp + soff[q] : sink) : sink;
      *reinterpret_cast<i32x4*>(dst) = stg[q];
    }
  };
  stage_load(1, -1);  // stored at step 0

  // ---- halo groups of this wave: rounds 0/1 are groups wid and wid + 8 with their X
  // fragments in VGPRs; round 2 (dilation-2 halos reach 17-19 groups at 33x33) goes to
  // the LAST waves (group 16 -> wave 7, 17 -> wave 6, ...), whose projection share is the
  // lighter one, with X in LDS
  auto hgroup = [&](int q) { return q < 2 ? wid + q * kSNW : 2 * kSNW + (kSNW - 1 - wid); };
  const int dummy = a.WR * a.WCP - 1;  // column >= W + 2*dil: never read by the depthwise
  bf16x8 xf[XR][KS];
  int hpos[XG];
  const bf16* inb = a.in + (size_t)b * HW * a.Cin;
  // branch-free so that every table and X load of the prologue is in flight at once
  // (padding lanes re-read the last halo entry and select zeros)
  int ent[XG];
#pragma unroll
  for (int q = 0; q < XG; ++q) ent[q] = tb[kHdr + min(hgroup(q) * 16 + r16, nh - 1)];
#pragma unroll
  for (int q = 0; q < XG; ++q) {
    const bool hv = hgroup(q) * 16 + r16 < nh;
    hpos[q] = hv ? (ent[q] & 4095) : dummy;
    const bf16* src = inb + (size_t)(ent[q] >> 12) * a.Cin + kq * 8;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const bf16x8 v = ld8(src + k * 32);
      if (q < XR) {
        xf[q < XR ? q : 0][k] = hv ? v : zero8();
      } else if (hgroup(q) < HG) {
        st8(reinterpret_cast<bf16*>(sX + ((kSNW - 1 - wid) * KS + k) * 1024 + lane * 16), hv ? v : zero8());
      }
    }
  }
#pragma unroll
  for (int q = 0; q < XR; ++q)
#pragma unroll
    for (int k = 0; k < KS; ++k) retire(xf[q][k]);

  // ---- depthwise output groups: og = wid, and og 8 (if any) on wave 1 (odd waves
  // carry the lighter projection share)
  int dpos[2];
  const int og1 = wid == 1 ? kSNW : kSOG;  // kSOG = none
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = p0 + (u == 0 ? wid : og1) * 16 + r16;
    dpos[u] = d * a.WCP + d;  // padding lanes: any in-window centre
    if (p < p1) {
      const int y = p / a.W, x = p - (p / a.W) * a.W;
      dpos[u] = (y - wy0) * a.WCP + x + d;
    }
  }
  const int toff_r = d * a.WCP;

  f32x4 acc[GPW][NSW];
#pragma unroll
  for (int g = 0; g < GPW; ++g)
#pragma unroll
    for (int n = 0; n < NSW; ++n) acc[g][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f16x8 h0 = {0, 0, 0, 0, 0, 0, 0, 0}, h6 = {6, 6, 6, 6, 6, 6, 6, 6};
  SPAN_STAMP(1);
  __syncthreads();
  SPAN_STAMP(2);

  // Step t: [C] chunk t-2, [A] chunk t, [B] chunk t-1. Every stage runs in every step
  // (no branches: the scheduler can issue all of a step's LDS reads up front); the
  // fill / drain steps compute on zeroed buffers or on stale finite data nobody reads.
  for (int t = 0; t < NC + 2; ++t) {
    const char* Dc = sD + (t & 1) * kSOG * 1024;          // [C] input
    const char* Wpc = sWp + (t & 1) * WPB;
    const char* Wec = sWe + (t & 1) * WEB;                // [A]
    const char* miscA = sMisc + (t % 3) * 1024;
    char* Et = sE + (t & 1) * 4 * PLANE;
    const char* miscB = sMisc + ((t + 2) % 3) * 1024;     // [B]: chunk t-1
    const char* ep = sE + ((t + 1) & 1) * 4 * PLANE + kq * PLANE;
    char* Dn = sD + ((t + 1) & 1) * kSOG * 1024;

    // ---- [C] projection of chunk t-2: acc[px, Cout slice] += Wp . D
    // The three stages touch disjoint buffers, so each wave may run them in any order:
    // waves 4-7 (the SIMD partners of waves 0-3) run [B] + staging first, so the LDS-heavy
    // depthwise of one wave overlaps the MFMA-heavy stages of its partner instead of all
    // eight waves hitting the LDS (then the matrix pipes) in lockstep.
    auto stage_C = [&]() {
    {
      f16x8 df[GPW];
#pragma unroll
      for (int g = 0; g < GPW; ++g) {
        const int og = pi + g * NPI;  // groups past OGn read zeroed slots: they were never written
        df[g] = og < kSOG ? *reinterpret_cast<const f16x8*>(Dc + og * 1024 + lane * 16) : h0;
      }
#pragma unroll
      for (int n = 0; n < NSW; ++n) {
        const f16x8 af = *reinterpret_cast<const f16x8*>(Wpc + (ci * NSW + n) * 1024 + lane * 16);
#pragma unroll
        for (int g = 0; g < GPW; ++g)
          if (pi + g * NPI < kSOG) acc[g][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, df[g], acc[g][n], 0, 0, 0);
      }
    }
    };
    auto stage_A = [&]() {
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const f32x4 be4 = *reinterpret_cast<const f32x4*>(miscA + 640 + (sub * 16 + kq * 4) * 4);
      char* eplane = Et + (sub * 2 + (kq >> 1)) * PLANE + (kq & 1) * 8;
      auto emit = [&](int q, const f32x4& e) {
        f16x4 o = {(f16)e[0], (f16)e[1], (f16)e[2], (f16)e[3]};
        o = __builtin_elementwise_min(__builtin_elementwise_max(o, h0.lo), h6.lo);
        *reinterpret_cast<f16x4*>(eplane + hpos[q] * 16) = o;
      };
      auto xfrag = [&](int q, int k) -> bf16x8 {
        return q < XR ? xf[q < XR ? q : 0][k]
                      : *reinterpret_cast<const bf16x8*>(sX + ((kSNW - 1 - wid) * KS + k) * 1024 + lane * 16);
      };
      if (TIGHT) {  // k-outer: one weight fragment live at a time
        f32x4 e[XG];
#pragma unroll
        for (int q = 0; q < XG; ++q) e[q] = be4;
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const bf16x8 wf = *reinterpret_cast<const bf16x8*>(Wec + (sub * KS + k) * 1024 + lane * 16);
#pragma unroll
          for (int q = 0; q < XG; ++q)
            if (hgroup(q) < HG) e[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xfrag(q, k), e[q], 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < XG; ++q)
          if (hgroup(q) < HG) emit(q, e[q]);
      } else {  // q-outer: one uniform branch per halo group, all KS fragments live
        bf16x8 wf[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k) wf[k] = *reinterpret_cast<const bf16x8*>(Wec + (sub * KS + k) * 1024 + lane * 16);
#pragma unroll
        for (int q = 0; q < XG; ++q) {
          if (hgroup(q) < HG) {
            f32x4 e = be4;
#pragma unroll
            for (int k = 0; k < KS; ++k) e = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[k], xfrag(q, k), e, 0, 0, 0);
            emit(q, e);
          }
        }
      }
    }
    };
    auto stage_B = [&]() {
    // (a 3-deep packed-FMA chain per row instead of 9)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int og = u == 0 ? wid : og1;
      if (og < OGn) {
        f16x8 sr[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          sr[r] = r == 0 ? *reinterpret_cast<const f16x8*>(miscB + 576 + kq * 16) : h0;
#pragma unroll
          for (int c3 = 0; c3 < 3; ++c3) {
            const int tp = r * 3 + c3;
            const f16x8 wt = *reinterpret_cast<const f16x8*>(miscB + tp * 64 + kq * 16);
            const int to = (r - 1) * toff_r + (c3 - 1) * d;
            sr[r] = *reinterpret_cast<const f16x8*>(ep + (dpos[u] + to) * 16) * wt + sr[r];
          }
        }
        f16x8 sv = sr[0] + sr[1] + sr[2];
        sv = __builtin_elementwise_min(__builtin_elementwise_max(sv, h0), h6);
        *reinterpret_cast<f16x8*>(Dn + og * 1024 + lane * 16) = sv;
      }
      if (TIGHT) __builtin_amdgcn_sched_barrier(0);
    }
    };
    auto stage_W = [&]() {
    // ---- commit the weights of step t+1 (We/misc of chunk t+1, Wp of chunk t-1) and
    // fetch those of step t+2; every slot written here was last read in step t-1
    stage_store(t + 1, t - 1);
#pragma unroll
    for (int q = 0; q < NLD; ++q) retire(stg[q]);
    stage_load(t + 2, t);
    };
    if (wid < 4) {
      stage_C();
      SPAN_STAMP(3 + 5 * t);
      if (TIGHT) __builtin_amdgcn_sched_barrier(0);
      stage_A();
      SPAN_STAMP(4 + 5 * t);
      if (TIGHT) __builtin_amdgcn_sched_barrier(0);
      stage_B();
      SPAN_STAMP(5 + 5 * t);
      stage_W();
    } else {
      stage_B();
      stage_W();
      if (TIGHT) __builtin_amdgcn_sched_barrier(0);
      stage_C();
      if (TIGHT) __builtin_amdgcn_sched_barrier(0);
      stage_A();
    }
    SPAN_STAMP(6 + 5 * t);
    __syncthreads();
    SPAN_STAMP(7 + 5 * t);
  }

  // ---- epilogue: + bias (+ residual), bf16; lane = 4 consecutive channels of one pixel.
  // Branch-free loads (padding lanes read pixel p0) so a group's bias / residual loads
  // are all in flight together; Cout % 16 == 0, so every subtile channel is real.
  bf16* outb = a.out + (size_t)b * HW * a.Cout;
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    if (pi + g * NPI >= OGn) continue;
    const int p = p0 + (pi + g * NPI) * 16 + r16;
    const bool pv = p < p1;
    const int pc = pv ? p : p0;
    f32x4 bb[NSW];
    bf16x4 rr[NSW];
#pragma unroll
    for (int n = 0; n < NSW; ++n) {
      const int co = (ci * NSW + n) * 16 + kq * 4;
      bb[n] = *reinterpret_cast<const f32x4*>(a.bp + co);
      rr[n] = a.residual ? *reinterpret_cast<const bf16x4*>(inb + (size_t)pc * a.Cin + co)
                         : bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
    }
#pragma unroll
    for (int n = 0; n < NSW; ++n) {
      const int co = (ci * NSW + n) * 16 + kq * 4;
      bf16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = (bf16)(acc[g][n][q] + bb[n][q] + (float)rr[n][q]);
      if (pv) *reinterpret_cast<bf16x4*>(outb + (size_t)p * a.Cout + co) = o;
    }
  }
  SPAN_STAMP(63);
}

template <int KS, int NS, int NPI, int XG>
void launch_span(const SpanArgs& a, hipStream_t st) {
  const size_t lds = fused_ir_span_lds(a.Cin, a.Cout, a.WR, a.WCP, XG > 2 ? a.xslots : 0);
  if (lds > 160 * 1024) throw std::invalid_argument("fused_ir_span: LDS over 160 KiB");
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_ir_span_kernel<KS, NS, NPI, XG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "fused_ir_span attr");
    attr = true;
  }
  hipLaunchKernelGGL((fused_ir_span_kernel<KS, NS, NPI, XG>), dim3(a.B * a.S), dim3(kSNT), lds, st, a);
  check_launch("fused_ir_span");
}

}  // namespace

size_t fused_ir_span_lds(int Cin, int Cout, int WR, int WCP, int xslots) {
  // We [2] + misc [3] + Wp [2] rings, E [2][4 planes], D [2][9 groups], third-round X
  const int KS = Cin / 32, NS = (Cout + 15) / 16;
  return (size_t)2 * 2 * KS * 1024 + 3 * 1024 + 2 * NS * 1024 + 8 * span_plane_bytes(WR, WCP) +
         2 * kSOG * 1024 + (size_t)xslots * KS * 1024 + 16;
}

void fused_ir_span(const FusedSpanParams& p, hipStream_t st) {
  if (p.Cin % 32 || p.Cout % 16 || p.hidP % 32 || p.hidP <= 0)
    throw std::invalid_argument("fused_ir_span: Cin % 32, Cout % 16, hidP % 32");
  if (p.residual && p.Cin != p.Cout) throw std::invalid_argument("fused_ir_span: residual needs Cin == Cout");
  if (p.dil < 1 || 2 * p.dil + 1 > 16 || p.WCP != p.W + 16 || p.WR < 2 * p.dil + 1 || p.WR * p.WCP > 4096)
    throw std::invalid_argument("fused_ir_span: bad window geometry");
  if (p.S < 1 || (p.H * p.W + p.S - 1) / p.S > kSOG * 16) throw std::invalid_argument("fused_ir_span: span > 144 px");
  if (p.H * p.W >= (1 << 19)) throw std::invalid_argument("fused_ir_span: map too large for the halo table");
  SpanArgs a{p.in, reinterpret_cast<const char*>(p.w), p.bp, p.table, p.out, p.B, p.H, p.W, p.Cin,
             p.Cout, p.hidP / 32, p.S, p.dil, p.residual, p.WCP, p.WR, p.hstride, p.xslots, p.trace};
  const int KS = p.Cin / 32, NS = p.Cout / 16;
  const int xg = p.xg, npi = p.npi;
  if (p.hstride < kHdr + xg * kSNW * 16) throw std::invalid_argument("fused_ir_span: halo table too short");
  if (p.xslots < 0 || p.xslots > kSNW || (xg < 3 && p.xslots > 0)) throw std::invalid_argument("fused_ir_span: bad xslots");
#define SPAN(K_, N_, P_, X_)                                     \
  if (KS == K_ && NS == N_ && npi == P_ && xg == X_) {           \
    launch_span<K_, N_, P_, X_>(a, st);                          \
    return;                                                      \
  }
  // blocks 7-9 (64->64), 10 (64->96), 11-12 (96->96), 13 (96->160), 14-15 (160->160),
  // 16 (160->320; NPI 4 would need > 256 VGPRs); xg 3 = dilation-2 halos
#define SPAN_X(K_, N_, P_) SPAN(K_, N_, P_, 2) SPAN(K_, N_, P_, 3)
  SPAN_X(2, 4, 2) SPAN_X(2, 4, 4) SPAN_X(2, 6, 4) SPAN_X(2, 6, 8) SPAN_X(3, 6, 4) SPAN_X(3, 6, 8)
  SPAN_X(3, 10, 4) SPAN_X(3, 10, 8) SPAN_X(5, 10, 4) SPAN_X(5, 10, 8) SPAN_X(5, 20, 2)
#undef SPAN_X
#undef SPAN
  throw std::invalid_argument("fused_ir_span: no instantiation for this (Cin, Cout, npi, xg)");
}

}  // namespace ssa
