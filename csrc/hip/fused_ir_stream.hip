// Fused MobileNetV2 inverted residual for the output-stride-16 stage, wave-specialised
// (blocks 7-15 of DeepLabv3-MobileNetV2 at 513^2: 33x33 maps, stride 1, dilation 1 or 2,
// hidden 384..960 channels), gfx950.
//
//   out = project( relu6( dw3x3_dil( relu6( expand(x) ) ) ) ) [+ x]
//
// The expanded tensor never leaves the CU (the reference runs the whole
// network as one Edge TPU call, /root/reference/sem_seg_server.py:162). Span
// decomposition, halo table and chunk images: ops/fused_span.py. The schedule replaced
// round 2's uniform-wave span kernel (every 32-channel step ~3,900 cycles against ~400
// cycles of MFMA work: each wave ran all three stages back to back with full lgkmcnt
// drains, staged weights through VGPRs with a vmcnt(0) drain per step, and spilled;
// profiles/r3_span_trace.txt).
//
// Both ReLU6 are a [0, 1] clamp here: the host packs the expansion / 6, the depthwise
// bias / 6 and the projection x 6 (fused_span.pack_fused_span), so the expansion's
// f32 -> f16 conversion and the last fma of the depthwise chain carry the clamp bit and
// no max / min instruction is issued (the depthwise was ~30 % of the VALU stream).
//
// Here:
//   * waves 0-3 ("A", one per SIMD) only EXPAND: chunk t of the hidden channels for the
//     span's halo pixels, X fragments resident in VGPRs (halo group a + 4q, q < 5),
//     E[t&1] (fp16, relu6) written to LDS octet planes (the span kernel's bank-conflict
//     free window layout);
//   * waves 4-7 ("BC", the SIMD partners of 3..0) run depthwise + projection of chunk
//     t-1: each lane computes the depthwise result for 8 channels of ONE output pixel --
//     exactly its B fragment of v_mfma_f32_16x16x32_f16 -- so D never touches LDS, and
//     accumulate [pixels x Cout] in fp32 VGPRs (output groups 3-b, 7-b, 11-b);
//   * the two roles run separate loops with the same barrier count, so the compiler
//     keeps X (A) and the accumulators (BC) in the same physical registers;
//   * chunk images (We fragments | Wp fragments | dw weights/biases, 1 KiB pieces) are
//     streamed by LDS-DMA (global_load_lds_dwordx4) into a 4-slot ring, two chunks
//     ahead; every wave waits only for its own pieces of the NEXT chunk (counted vmcnt)
//     before the step's single s_barrier (no __syncthreads: its fence drains vmcnt).
// One step = one barrier; the matrix pipe of each SIMD is shared by an expansion wave
// (MFMA-heavy) and a depthwise+projection wave (VALU/LDS-heavy + MFMA), so one wave's
// LDS latency hides under the other's MFMAs.
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

typedef _Float16 f16;
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// waves per workgroup: 8 (4 expansion + 4 depthwise/projection) or, for the MODE-2
// variant, 12 (4 + 8: two depthwise/projection waves per SIMD hide each other's LDS and
// VALU latency -- the same lever that took the grouped ASPP GEMM from 8 to 16 waves)
__host__ __device__ constexpr int stream_waves(int mode) { return (mode & 3) == 2 ? 12 : 8; }
constexpr int kHdr = 4;    // span table header: p0, p1, wy0, nh
constexpr int kXQ = 5;     // halo groups per expansion wave (<= 20 groups = 320 halo px)
constexpr int kGB = 3;     // output groups per depthwise+projection wave (<= 12 groups)
constexpr int kSpanPx = 9 * 16;  // output pixels per span at most (4 waves x 2 groups + group 8)
// chunk-image ring slots: 4 (DMA two chunks ahead) or, for Cout 320 (31 KiB chunk images), 3
__host__ __device__ constexpr int stream_nsl(int NS) { return NS > 10 ? 3 : 4; }
// epilogue passes over Cout (the fp32 output tile of a 144-pixel span at Cout 320 would
// need 186 KiB of LDS)
__host__ __device__ constexpr int stream_npass(int NS) { return NS > 10 ? 2 : 1; }

struct StreamArgs {
  const bf16* in; const char* w; const float* bp; const int* table; bf16* out;
  int B, H, W, Cin, Cout, NC, S, dil, residual, WCP, WR, hstride;
  long long* trace;  // debug: s_memtime stamps [block][wave 0 / 4][64], nullptr normally
  int HS;            // hidden splits: workgroups per span, each a contiguous range of chunks
  float* part;       // HS > 1: fp32 projection partials [HS][B * H * W][Cout] (no bias)
  int* cnt;          // HS > 1, in-launch combine: per-span arrival tickets [B * S] (zero between
                     // launches: the last arriver resets its word), else null (stream_combine)
};

// Debug timeline (a.trace != nullptr): lane 0 of waves 0 (expansion) and 4 (its SIMD
// partner's role, depthwise+projection) stamps s_memtime (vector stores to the trace buffer)
#define STREAM_STAMP(slot)                                                                           \
  do {                                                                                               \
    if (a.trace && (wid == 0 || wid == 4) && lane == 0 && (slot) < 64)                               \
      a.trace[((size_t)blockIdx.x * 2 + (wid >> 2)) * 64 + (slot)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

__host__ __device__ inline int stream_plane_bytes(int WR, int WCP) { return (WR * WCP + 15) / 16 * 16 * 16; }

__device__ __forceinline__ void wait_vm(int n) {
  // n is wave-uniform; a counted wait leaves the newer chunk's DMA pieces in flight
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void step_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes landed
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- expansion of one chunk for NQ halo rounds (compile-time: no branches inside)
template <int KS, int NQ, int NR>
__device__ __forceinline__ void expand_chunk(const char* Wc, const char* misc, char* Eb, int PLANE,
                                             const f32x4 (&R)[NR], const int (&hpos)[kXQ],
                                             int lane, int kq) {
  const f16x4 z4 = {0, 0, 0, 0}, s4 = {1, 1, 1, 1};  // folded ReLU6: v_cvt_pk_f16_f32 ... clamp
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
    const f32x4 be4 = *reinterpret_cast<const f32x4*>(misc + 640 + (sub * 16 + kq * 4) * 4);
    bf16x8 wf[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) wf[k] = *reinterpret_cast<const bf16x8*>(Wc + (sub * KS + k) * 1024 + lane * 16);
    f32x4 e[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) e[q] = be4;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int q = 0; q < NQ; ++q) e[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[k], __builtin_bit_cast(bf16x8, R[q * KS + k]), e[q], 0, 0, 0);
    char* ep = Eb + (sub * 2 + (kq >> 1)) * PLANE + (kq & 1) * 8;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      f16x4 o = {(f16)e[q][0], (f16)e[q][1], (f16)e[q][2], (f16)e[q][3]};
      o = __builtin_elementwise_min(__builtin_elementwise_max(o, z4), s4);
      *reinterpret_cast<f16x4*>(ep + hpos[q] * 16) = o;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---- depthwise 3x3 of one output pixel x 8 channels: ONE fma chain per channel pair over
// the 9 taps, starting from the (scaled) bias; the clamp of its last fma is the folded ReLU6
__device__ __forceinline__ f16x8 dw_chain(const f16x8 (&v)[9], const f16x8 (&wt)[9], f16x8 bd) {
  const f16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0}, o8 = {1, 1, 1, 1, 1, 1, 1, 1};
  f16x8 r = bd;
#pragma unroll
  for (int t = 0; t < 9; ++t) r = v[t] * wt[t] + r;
  return __builtin_elementwise_min(__builtin_elementwise_max(r, z8), o8);
}

// ---- depthwise + projection of one chunk: output groups g0, g1 over all NS Cout subtiles
// and g2 over NS3 subtiles starting at n3 (NS3 = NS / 2 for the wide blocks: the ninth
// group of a span is split over two waves so the accumulators fit 256 VGPRs).
// Tap offsets are template constants (dilation, window pitch): the 9 taps of a group are
// one base VGPR + ds_read immediates, not 27 loop-invariant addresses.
template <int NS, int NS3, int DIL, int WCP, int NR, bool PIPE>
__device__ __forceinline__ void dwproj_chunk(const char* Wp, const char* misc, const char* Ek,
                                             const int (&dpos)[kGB], int n3, f32x4 (&R)[NR],
                                             int lane, int kq) {
  f16x8 wt[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wt[t] = *reinterpret_cast<const f16x8*>(misc + t * 64 + kq * 16);
  const f16x8 bd = *reinterpret_cast<const f16x8*>(misc + 576 + kq * 16);
  auto taps = [&](int g, f16x8 (&v)[9]) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
      v[t] = *reinterpret_cast<const f16x8*>(Ek + dpos[g] * 16 + ((t / 3 - 1) * DIL * WCP + (t % 3 - 1) * DIL) * 16);
  };
  auto dw = [&](const f16x8 (&v)[9]) { return dw_chain(v, wt, bd); };
  f16x8 dv[kGB];
  if (PIPE) {
    // the next group's 9 taps are in flight while this group's depthwise runs (the
    // timeline of the unpipelined form: ~2,600 cycles per step, LDS latency exposed 3x)
    f16x8 va[9], vb[9];
    taps(0, va);
    __builtin_amdgcn_sched_barrier(0);
    taps(1, vb);
    dv[0] = dw(va);
    __builtin_amdgcn_sched_barrier(0);
    taps(2, va);
    dv[1] = dw(vb);
    __builtin_amdgcn_sched_barrier(0);
    dv[2] = dw(va);
  } else {
#pragma unroll
    for (int g = 0; g < kGB; ++g) {
      f16x8 v[9];
      taps(g, v);
      dv[g] = dw(v);
      __builtin_amdgcn_sched_barrier(0);  // one group's 9 taps live at a time (VGPR budget)
    }
  }
#pragma unroll
  for (int n = 0; n < NS; ++n) {
    const f16x8 af = *reinterpret_cast<const f16x8*>(Wp + n * 1024 + lane * 16);
    R[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, dv[0], R[n], 0, 0, 0);
    R[NS + n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, dv[1], R[NS + n], 0, 0, 0);
    if (NS3 == NS) R[2 * NS + n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, dv[2], R[2 * NS + n], 0, 0, 0);
  }
  if (NS3 != NS) {
#pragma unroll
    for (int n = 0; n < NS3; ++n) {
      const f16x8 af = *reinterpret_cast<const f16x8*>(Wp + (n3 + n) * 1024 + lane * 16);
      R[2 * NS + n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, dv[2], R[2 * NS + n], 0, 0, 0);
    }
  }
}

// ---- generic form: NG output groups (taps at dpos[g]) x NN Cout subtiles starting at n0
// (indices past nlast clamp to it: duplicated work that is never stored), accumulating
// into R[r0 + g * NN + j]. Used with group 8 moved to the expansion waves (G8A): those run
// one group x ceil(NS/4) subtiles each, the projection waves two groups x NS.
template <int NG, int NN, int DIL, int WCP, int NR, bool PIPE = true, bool HALF = false>
__device__ __forceinline__ void dwproj_groups(const char* Wp, const char* misc, const char* Ek,
                                              const int (&dpos)[NG], int n0, int nlast, f32x4 (&R)[NR],
                                              int r0, int lane, int kq) {
  f16x8 dv[NG];
  if (HALF) {
    // register-lean form for the kernels whose accumulators take 160 VGPRs (block 16, and
    // the G8A variants of blocks 14-15: those spilled, and each spill reload's vmcnt(0)
    // also waited for the next chunk's LDS-DMA): the 8 channels in two f16x4 halves, so
    // only half the tap and weight registers are live at a time (same LDS bytes)
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const h4 z4 = {0, 0, 0, 0}, o4 = {1, 1, 1, 1};
    h4 lo[NG], hi[NG];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      h4 wt[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) wt[t] = *reinterpret_cast<const h4*>(misc + t * 64 + kq * 16 + hf * 8);
      const h4 bd = *reinterpret_cast<const h4*>(misc + 576 + kq * 16 + hf * 8);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        h4 v[9];
#pragma unroll
        for (int t = 0; t < 9; ++t)
          v[t] = *reinterpret_cast<const h4*>(Ek + dpos[g] * 16 + hf * 8 +
                                              ((t / 3 - 1) * DIL * WCP + (t % 3 - 1) * DIL) * 16);
        h4 r = bd;
#pragma unroll
        for (int t = 0; t < 9; ++t) r = v[t] * wt[t] + r;
        r = __builtin_elementwise_min(__builtin_elementwise_max(r, z4), o4);
        if (hf == 0) lo[g] = r; else hi[g] = r;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) dv[g] = __builtin_shufflevector(lo[g], hi[g], 0, 1, 2, 3, 4, 5, 6, 7);
  } else {
    f16x8 wt[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[t] = *reinterpret_cast<const f16x8*>(misc + t * 64 + kq * 16);
    const f16x8 bd = *reinterpret_cast<const f16x8*>(misc + 576 + kq * 16);
    auto taps = [&](int g, f16x8 (&v)[9]) {
#pragma unroll
      for (int t = 0; t < 9; ++t)
        v[t] = *reinterpret_cast<const f16x8*>(Ek + dpos[g] * 16 + ((t / 3 - 1) * DIL * WCP + (t % 3 - 1) * DIL) * 16);
    };
    auto dw = [&](const f16x8 (&v)[9]) { return dw_chain(v, wt, bd); };
    if (NG == 2 && PIPE) {  // the second group's taps in flight while the first one's depthwise runs
      f16x8 va[9], vb[9];
      taps(0, va);
      __builtin_amdgcn_sched_barrier(0);
      taps(NG - 1, vb);
      dv[0] = dw(va);
      dv[NG - 1] = dw(vb);
    } else {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        f16x8 v[9];
        taps(g, v);
        dv[g] = dw(v);
        if (NG > 1) __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    const int n = min(n0 + j, nlast);
    const f16x8 af = *reinterpret_cast<const f16x8*>(Wp + n * 1024 + lane * 16);
#pragma unroll
    for (int g = 0; g < NG; ++g)
      R[r0 + g * NN + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, dv[g], R[r0 + g * NN + j], 0, 0, 0);
    // register-lean: at most 4 projection fragments in flight (the scheduler otherwise
    // hoists all NN fragment reads above the first MFMA: 80 VGPRs at NN = 20)
    if (HALF && j % 4 == 3) __builtin_amdgcn_sched_barrier(0);
  }
}

// slabs the in-launch combine loads per round trip
constexpr int kCombineHS = 8;

template <int KS, int NS, int XQ, int DIL, int WCP, int MODE>
__global__ __launch_bounds__(64 * stream_waves(MODE)) void fused_ir_stream_kernel(StreamArgs a) {
  // MODE 0: 8 waves, the ninth output group split over the projection waves;
  // 1 (G8A): 8 waves, the ninth group on the expansion waves; 2: 12 waves, projection
  // wave b owns group b, wave 7 also the ninth group
  // MODE & 4: a 3-slot chunk ring (one chunk of DMA lookahead) for the blocks whose default is
  // 4 slots: 72 instead of 81 KiB for blocks 7-9, so two workgroups -- of one plan copy or of
  // two slots' concurrent steps -- can share a CU's 160 KiB of LDS
  constexpr bool G8A = (MODE & 3) == 1;
  // MODE & 8: lattice spans (ops/fused_span.lattice_table): a dilation-2 layer run on the
  // phase-class lattice, where its taps are dilation-1 taps (DIL = 1 here) and a span's halo
  // is +- 1 lattice row: 1.22x instead of 1.87x of the output pixels expanded at 33^2, S = 8.
  // The span's output pixels and their window centres come from the table's output list;
  // p0 = 0 and p1 = the span's length, so "span pixel" px is output-list entry px.
  constexpr bool LAT = (MODE & 8) != 0;
  __shared__ int s_opix[LAT ? kSpanPx : 1];  // output-list pixel indices (epilogue)
  constexpr int kNW = stream_waves(MODE), kNT = 64 * kNW;
  constexpr int NPC = 2 * KS + NS + 1;          // 1 KiB pieces per chunk image
  constexpr int CHB = NPC * 1024;
  constexpr int WEB = 2 * KS * 1024, WPB = NS * 1024;
  constexpr int kNSL = (MODE & 4) ? 3 : stream_nsl(NS);
  constexpr int LAG = kNSL - 2;
  // every wave issues MP pieces per chunk (the last piece duplicated where NPC % 8 != 0:
  // identical bytes to the same slot), so the counted waits are compile-time constants
  constexpr int MP = (NPC + kNW - 1) / kNW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int PLANE = stream_plane_bytes(a.WR, WCP);
  char* ring = smem;                   // [kNSL][CHB]
  char* sE = smem + kNSL * CHB;        // [2][4 octet planes][PLANE]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  // block -> (image b, span j, hidden slice hs); the HS slices of a span are adjacent
  const int hs = blockIdx.x % a.HS, bj = blockIdx.x / a.HS;
  const int b = bj / a.S, j = bj - (bj / a.S) * a.S;
  const int* tb = a.table + (size_t)j * a.hstride;
  const int p0 = tb[0], p1 = tb[1], wy0 = tb[2], nh = tb[3];
  const int HW = a.H * a.W, d = DIL;
  // this workgroup's chunks [cb, cb + NC): batch 1 has B * S = 16..32 workgroups for 256
  // CUs, so the hidden chunks of a span are split over HS workgroups whose fp32 partial
  // projections stream_combine sums (+ bias, residual) in a fixed order
  const int cb = hs * a.NC / a.HS, NC = (hs + 1) * a.NC / a.HS - cb;
  const char* wsrc = a.w + (size_t)cb * CHB;
  const bf16* inb = a.in + (size_t)b * HW * a.Cin;

  auto issue = [&](int c) {
    const char* src = wsrc + (size_t)c * CHB + lane * 16;
    char* dst = ring + (c % kNSL) * CHB;
#pragma unroll
    for (int q = 0; q < MP; ++q) {
      const int piece = min(wid + q * kNW, NPC - 1);
      __builtin_amdgcn_global_load_lds(src + piece * 1024, (lds_ptr_t)(dst + piece * 1024), 16, 0, 0);
    }
  };
  // end of step t: chunk t+1 must have landed; chunk t+LAG (issued this step) may fly on

  // ---- prologue: X fragments (A waves), first LAG chunk images, E zeroed (padding taps)
  const int dummy = a.WR * WCP - 1;  // window slot never read by the depthwise
  const int olist = a.hstride - kSpanPx;  // LAT: output list offset in the span's row
  if (LAT)
    for (int i = tid; i < p1 - p0; i += kNT) s_opix[i] = tb[olist + i] >> 12;  // visible after the prologue barrier
  // ONE register array for both roles: the expansion waves keep their X fragments in it,
  // the depthwise+projection waves their fp32 accumulators (the allocator does not share
  // two role-private arrays by itself: 190..256 VGPRs + spills against max(A, BC))
  constexpr int NS3 = NS >= 10 ? NS / 2 : NS;
  constexpr int Q8 = (NS + 3) / 4;  // G8A: group-8 subtiles per expansion wave
  constexpr int NRA = XQ * KS + (G8A ? Q8 : 0), NRB = (G8A || (MODE & 3) == 2) ? 2 * NS : 2 * NS + NS3;
  constexpr int NR = NRA > NRB ? NRA : NRB;
  // G8A with >= 112 accumulator / X VGPRs: the register-lean depthwise (dwproj_groups HALF)
  constexpr bool LEAN = G8A && NR >= 28;
  f32x4 R[NR];
  int hpos[kXQ];
  if (wid < 4) {
    int ent[XQ];
#pragma unroll
    for (int q = 0; q < XQ; ++q) ent[q] = tb[kHdr + min((wid + 4 * q) * 16 + r16, nh - 1)];
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const bool hv = (wid + 4 * q) * 16 + r16 < nh;
      hpos[q] = hv ? (ent[q] & 4095) : dummy;
      const bf16* src = inb + (size_t)(ent[q] >> 12) * a.Cin + kq * 8;
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const bf16x8 v = ld8(src + k * 32);
        R[q * KS + k] = __builtin_bit_cast(f32x4, hv ? v : zero8());
      }
    }
  }
#pragma unroll
  for (int c = 0; c < LAG; ++c)
    if (c < NC) issue(c);
  for (int i = tid; i < 8 * PLANE / 16; i += kNT) *reinterpret_cast<i32x4*>(sE + i * 16) = i32x4{0, 0, 0, 0};
  // chunk 0 (and the X loads, issued earlier) landed; chunk 1 may stay in flight
  STREAM_STAMP(0);
  if (LAG < NC) wait_vm(MP * (LAG - 1));
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  step_barrier();
  STREAM_STAMP(1);

  // ONE loop for both roles, R carried around it: the loop-header phi is what makes the
  // register allocator keep the expansion waves' X fragments and the projection waves'
  // accumulators in the same VGPRs (two role-private loops got the sum of both roles'
  // registers, 190..256 VGPRs + spills, instead of the max).
  // Step t: expansion waves expand chunk t (t < NC); depthwise+projection waves run chunk
  // t-1 (t >= 1). Wave bw = wid - 4 of the latter (the SIMD partner of expansion wave
  // 3 - bw) owns output groups 3-bw and 7-bw over all Cout subtiles, and group 8 (the ninth
  // 16-pixel group of a 129..144 pixel span) over subtiles [n3, n3 + NS3): waves bw 0/1
  // split it for the wide blocks, waves 2/3 compute a copy that is never stored.
  const bool expander = wid < 4;
  const int bw = wid - 4;
  const int og[kGB] = {(MODE & 3) == 2 ? bw : 3 - bw, (MODE & 3) == 2 ? 8 : 7 - bw, 8};
  const int n3 = NS3 == NS ? 0 : (bw & 1) * NS3;
  const bool own3 = NS3 == NS ? bw == 0 : bw < 2;
  int dpos[kGB];
#pragma unroll
  for (int g = 0; g < kGB; ++g) {
    const int p = p0 + (expander ? 8 : og[g]) * 16 + r16;  // G8A: expansion waves own group 8
    dpos[g] = d * WCP + d;  // padding lanes: any in-window centre
    if (p < p1) {
      if (LAT) {
        dpos[g] = tb[olist + p] & 4095;
      } else {
        const int y = p / a.W, x = p - (p / a.W) * a.W;
        dpos[g] = (y - wy0) * WCP + x + d;
      }
    }
  }
  const int dpos8[1] = {dpos[0]};
  const int dpos01[2] = {dpos[0], dpos[1]};
  if (!expander) {
#pragma unroll
    for (int n = 0; n < NR; ++n) R[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else if (G8A) {
#pragma unroll
    for (int j = 0; j < Q8; ++j) R[XQ * KS + j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int t = 0; t <= NC; ++t) {
    const bool more = t + LAG < NC;
    if (more) issue(t + LAG);
    if (expander) {
      if (G8A && !(LEAN && NS > 10)) {
        // group 8 of chunk t-1: its 9 taps, weights and bias are read FIRST, so their LDS
        // latency runs under the expansion's MFMAs instead of after them
        f16x8 v8[9], wt8[9], bd8 = {};
        const int c = t - 1;
        if (t >= 1) {
          const char* misc = ring + (c % kNSL) * CHB + WEB + WPB;
          const char* Ek = sE + (c & 1) * 4 * PLANE + kq * PLANE;
#pragma unroll
          for (int u = 0; u < 9; ++u) {
            wt8[u] = *reinterpret_cast<const f16x8*>(misc + u * 64 + kq * 16);
            v8[u] = *reinterpret_cast<const f16x8*>(Ek + dpos8[0] * 16 + ((u / 3 - 1) * DIL * WCP + (u % 3 - 1) * DIL) * 16);
          }
          bd8 = *reinterpret_cast<const f16x8*>(misc + 576 + kq * 16);
        }
        if (t < NC) {
          const char* Wc = ring + (t % kNSL) * CHB;
          expand_chunk<KS, XQ, NR>(Wc, Wc + WEB + WPB, sE + (t & 1) * 4 * PLANE, PLANE, R, hpos, lane, kq);
        }
        if (t >= 1) {
          const char* Wp = ring + (c % kNSL) * CHB + WEB;
          const f16x8 dv = dw_chain(v8, wt8, bd8);
#pragma unroll
          for (int j = 0; j < Q8; ++j) {
            const int n = min(wid * Q8 + j, NS - 1);
            const f16x8 af = *reinterpret_cast<const f16x8*>(Wp + n * 1024 + lane * 16);
            R[XQ * KS + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, dv, R[XQ * KS + j], 0, 0, 0);
          }
        }
      } else {
      if (t < NC) {
        const char* Wc = ring + (t % kNSL) * CHB;
        expand_chunk<KS, XQ, NR>(Wc, Wc + WEB + WPB, sE + (t & 1) * 4 * PLANE, PLANE, R, hpos, lane, kq);
      }
      if (G8A && t >= 1) {
        const int c = t - 1;
        const char* Wp = ring + (c % kNSL) * CHB + WEB;
        dwproj_groups<1, Q8, DIL, WCP, NR, true, (LEAN && NS > 10)>(Wp, Wp + WPB, sE + (c & 1) * 4 * PLANE + kq * PLANE, dpos8,
                                           wid * Q8, NS - 1, R, XQ * KS, lane, kq);
      }
      }
    } else if (t >= 1) {
      const int c = t - 1;
      const char* Wp = ring + (c % kNSL) * CHB + WEB;
      if ((MODE & 3) == 2) {
        const char* Ek = sE + (c & 1) * 4 * PLANE + kq * PLANE;
        // Cout 160 (lattice blocks 14-15): the register-lean depthwise, so 12 waves fit 168 VGPRs
        dwproj_groups<1, NS, DIL, WCP, NR, true, (NS > 6)>(Wp, Wp + WPB, Ek, dpos8, 0, NS - 1, R, 0, lane, kq);
        if (bw == 7) {
          const int dposn[1] = {dpos[1]};
          dwproj_groups<1, NS, DIL, WCP, NR, true, (NS > 6)>(Wp, Wp + WPB, Ek, dposn, 0, NS - 1, R, NS, lane, kq);
        }
      } else if (G8A)
        dwproj_groups<2, NS, DIL, WCP, NR, (NS <= 10 && !LEAN), (LEAN && NS > 10)>(Wp, Wp + WPB, sE + (c & 1) * 4 * PLANE + kq * PLANE, dpos01, 0,
                                           NS - 1, R, 0, lane, kq);
      else
        dwproj_chunk<NS, NS3, DIL, WCP, NR, true>(Wp, Wp + WPB, sE + (c & 1) * 4 * PLANE + kq * PLANE,
                                                  dpos, n3, R, lane, kq);
    }
    STREAM_STAMP(2 + 3 * t);
    // end of step t: chunk t+1 landed; chunk t+LAG (issued this step) may fly on
    if (more) wait_vm(MP * (LAG - 1));
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STREAM_STAMP(3 + 3 * t);
    step_barrier();
    STREAM_STAMP(4 + 3 * t);
  }
  // ---- epilogue, per pass over a Cout slice [h * NSP, (h + 1) * NSP) subtiles:
  // part 1, accumulators -> fp32 output tile [span pixel][slice] in LDS (ring and E are
  // free: every DMA was waited for and every read is behind the last barrier); a row pitch
  // of slice + 4 floats keeps the 16 pixel rows of a ds_write_b128 lane group on distinct
  // banks. Part 2 (all waves): + bias (+ residual), bf16, fully coalesced 16-byte stores of
  // the span's contiguous output rows (the per-fragment 8-byte stores of the first version
  // took 5-21k cycles per workgroup: 16 pixels x 32 B segments per store instruction).
  STREAM_STAMP(62);
  constexpr int NPASS = stream_npass(NS), NSP = NS / NPASS;
  float* O = reinterpret_cast<float*>(smem);
  const int OS = NSP * 16 + 4;
#pragma unroll
  for (int h = 0; h < NPASS; ++h) {
    if (h > 0) step_barrier();  // the previous pass's tile has been copied out
    if (!expander) {
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int n = 0; n < NS; ++n)
          if (n / NSP == h && ((MODE & 3) != 2 || g == 0 || bw == 7))
            *reinterpret_cast<f32x4*>(O + (og[g] * 16 + r16) * OS + (n - h * NSP) * 16 + kq * 4) = R[g * NS + n];
      if (own3 && (MODE & 3) == 0) {
#pragma unroll
        for (int n = 0; n < NS3; ++n)
          if ((n3 + n) / NSP == h)
            *reinterpret_cast<f32x4*>(O + (og[2] * 16 + r16) * OS + (n3 + n - h * NSP) * 16 + kq * 4) = R[2 * NS + n];
      }
    } else if (G8A) {
#pragma unroll
      for (int j = 0; j < Q8; ++j) {
        const int n = wid * Q8 + j;
        if (n < NS && n / NSP == h)
          *reinterpret_cast<f32x4*>(O + (8 * 16 + r16) * OS + (n - h * NSP) * 16 + kq * 4) = R[XQ * KS + j];
      }
    }
    step_barrier();
    const int C8 = NSP * 2, c0 = h * NSP * 16;  // 8-channel units per pixel in the slice
    const int units = (p1 - p0) * C8;
    if (a.HS > 1) {  // fp32 partial of this hidden slice, bias / residual added by the combine
      float* pb = a.part + ((size_t)hs * a.B * HW + (size_t)b * HW) * a.Cout + c0;
      for (int u = tid; u < units; u += kNT) {
        const int px = u / C8, c = (u - px * C8) * 8;
        float* q = pb + (size_t)(LAT ? s_opix[px] : p0 + px) * a.Cout + c;
        *reinterpret_cast<f32x4*>(q) = *reinterpret_cast<const f32x4*>(O + px * OS + c);
        *reinterpret_cast<f32x4*>(q + 4) = *reinterpret_cast<const f32x4*>(O + px * OS + c + 4);
      }
      continue;
    }
    bf16* outb = a.out + (size_t)b * HW * a.Cout + c0;
    const bf16* resb = inb + c0;
    for (int u = tid; u < units; u += kNT) {
      const int px = u / C8, c = (u - px * C8) * 8;
      const int gp = LAT ? s_opix[px] : p0 + px;  // the pixel's index in the image
      const f32x4 o0 = *reinterpret_cast<const f32x4*>(O + px * OS + c);
      const f32x4 o1 = *reinterpret_cast<const f32x4*>(O + px * OS + c + 4);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.bp + c0 + c);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(a.bp + c0 + c + 4);
      bf16x8 r = zero8();
      if (a.residual) r = ld8(resb + (size_t)gp * a.Cin + c);
      bf16x8 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        o[q] = (bf16)(o0[q] + b0[q] + (float)r[q]);
        o[q + 4] = (bf16)(o1[q] + b1[q] + (float)r[q + 4]);
      }
      st8(outb + (size_t)gp * a.Cout + c, o);
    }
  }
  if (a.HS > 1 && a.cnt) {
    // in-launch combine (cdna_hip_programming.md, split-K reduction recipe): every wave
    // drains its partial stores, one lane releases them at agent scope and draws a ticket;
    // the span's last arriver acquires, resets the ticket and sums the HS slabs in the
    // fixed order h = 0..HS-1 (+ bias, residual) into the bf16 output -- the stream_combine
    // launch (4.5-5.6 us per block at batch 1, profiles/r4_b1_layer_times.txt) disappears
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's partial stores drained; O is no longer read
    int* s_flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int t = __hip_atomic_fetch_add(a.cnt + bj, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == a.HS - 1;
      if (last) {
        __hip_atomic_store(a.cnt + bj, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *s_flag = last;
    }
    __syncthreads();
    if (*reinterpret_cast<volatile int*>(s_flag)) {
      const int C8 = a.Cout / 8, units = (p1 - p0) * C8;
      const size_t slab = (size_t)a.B * HW * a.Cout;
      const float* pb = a.part + (size_t)b * HW * a.Cout;
      bf16* outb = a.out + (size_t)b * HW * a.Cout;
      const bf16* resb = inb;
      for (int u = tid; u < units; u += kNT) {
        const int px = u / C8, c = (u - px * C8) * 8;
        const int gp = LAT ? s_opix[px] : p0 + px;
        f32x4 s0 = *reinterpret_cast<const f32x4*>(a.bp + c), s1 = *reinterpret_cast<const f32x4*>(a.bp + c + 4);
        const float* q = pb + (size_t)gp * a.Cout + c;
        // the slabs' loads (and the residual's) issued kCombineHS at a time before their adds:
        // one L2 round trip per group instead of one per slab (as stream_combine_kernel's HSM
        // form; slabs past HS re-read the last one and are not added; order h = 0..HS-1)
        bf16x8 r = zero8();
        if (a.residual) r = ld8(resb + (size_t)gp * a.Cin + c);
        for (int h0 = 0; h0 < a.HS; h0 += kCombineHS) {
          f32x4 v0[kCombineHS], v1[kCombineHS];
#pragma unroll
          for (int h = 0; h < kCombineHS; ++h) {
            const size_t o = (size_t)(h0 + h < a.HS ? h0 + h : a.HS - 1) * slab;
            v0[h] = *reinterpret_cast<const f32x4*>(q + o);
            v1[h] = *reinterpret_cast<const f32x4*>(q + o + 4);
          }
#pragma unroll
          for (int h = 0; h < kCombineHS; ++h)
            if (h0 + h < a.HS) {
              s0 += v0[h];
              s1 += v1[h];
            }
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = (bf16)(s0[e] + (float)r[e]);
          o[e + 4] = (bf16)(s1[e] + (float)r[e + 4]);
        }
        st8(outb + (size_t)gp * a.Cout + c, o);
      }
    }
  }
  STREAM_STAMP(63);
}

template <int KS, int NS, int XQ, int DIL, int WCP, int MODE>
void launch_stream(const StreamArgs& a, hipStream_t st) {
  const size_t lds = fused_ir_stream_lds(a.Cin, a.Cout, a.WR, a.WCP, (MODE & 4) ? 3 : 0);
  // the lattice form's static output-list array (s_opix) shares the CU's 160 KiB
  constexpr size_t kStatic = (MODE & 8) ? kSpanPx * sizeof(int) : 64;
  if (lds > 160 * 1024 - kStatic) throw std::invalid_argument("fused_ir_stream: LDS over 160 KiB");
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_ir_stream_kernel<KS, NS, XQ, DIL, WCP, MODE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - kStatic),
          "fused_ir_stream attr");
    attr = true;
  }
  hipLaunchKernelGGL((fused_ir_stream_kernel<KS, NS, XQ, DIL, WCP, MODE>), dim3(a.B * a.S * a.HS),
                     dim3(64 * stream_waves(MODE)), lds, st, a);
  check_launch("fused_ir_stream");
}

}  // namespace

size_t fused_ir_stream_lds(int Cin, int Cout, int WR, int WCP, int nsl) {
  const int KS = Cin / 32, NS = (Cout + 15) / 16;
  const size_t main = (size_t)(nsl > 0 ? nsl : stream_nsl(NS)) * (2 * KS + NS + 1) * 1024 +
                      8 * (size_t)stream_plane_bytes(WR, WCP);
  const size_t otile = (size_t)kGB * 4 * 16 * (NS / stream_npass(NS) * 16 + 4) * 4;  // epilogue tile
  return main > otile ? main : otile;
}

void fused_ir_stream(const FusedSpanParams& p, hipStream_t st) {
  if (p.Cin % 32 || p.Cout % 16 || p.hidP % 32 || p.hidP <= 0)
    throw std::invalid_argument("fused_ir_stream: Cin % 32, Cout % 16, hidP % 32");
  if (p.residual && p.Cin != p.Cout) throw std::invalid_argument("fused_ir_stream: residual needs Cin == Cout");
  const bool lat = (p.npi & 8) != 0;  // lattice spans (dilation 2 as dilation-1 taps)
  if (lat ? (p.dil != 2 || p.WCP != (p.W + 1) / 2 + 3 || p.WR < 3 || p.WR * p.WCP > 4096)
          : (p.dil < 1 || 2 * p.dil + 1 > 16 || p.WCP != p.W + 16 || p.WR < 2 * p.dil + 1 || p.WR * p.WCP > 4096))
    throw std::invalid_argument("fused_ir_stream: bad window geometry");
  if (lat && (p.hstride < kHdr + kSpanPx || p.nh_max > 3 * 64))
    throw std::invalid_argument("fused_ir_stream: lattice table needs an output list and <= 192 halo px");
  if (p.S < 1 || (p.H * p.W + p.S - 1) / p.S > kGB * 4 * 16) throw std::invalid_argument("fused_ir_stream: span too long");
  if (p.H * p.W >= (1 << 19)) throw std::invalid_argument("fused_ir_stream: map too large for the halo table");
  if (p.nh_max > kXQ * 4 * 16) throw std::invalid_argument("fused_ir_stream: halo over 320 pixels");
  if (p.hsplit < 1 || p.hsplit > p.hidP / 32 || (p.hsplit > 1 && p.part == nullptr))
    throw std::invalid_argument("fused_ir_stream: hsplit in [1, hidP / 32], partials buffer for hsplit > 1");
  StreamArgs a{p.in, reinterpret_cast<const char*>(p.w), p.bp, p.table, p.out, p.B, p.H, p.W, p.Cin,
               p.Cout, p.hidP / 32, p.S, p.dil, p.residual, p.WCP, p.WR, p.hstride, p.trace,
               p.hsplit, p.part, p.hsplit > 1 ? p.cnt : nullptr};
  const int KS = p.Cin / 32, NS = p.Cout / 16;
  // instantiated for the 33-wide maps of the headline (window pitch W + 16 = 49) at
  // dilation 1 (halo <= 16 groups: 4 rounds per expansion wave) and 2 (<= 20: 5 rounds)
  if (p.W != 33 || p.dil > 2 || p.nh_max > (p.dil == 1 ? 4 : 5) * 64)
    throw std::invalid_argument("fused_ir_stream: W 33, dilation 1/2, halo <= 256/320 px");
  // an unknown variant, or the 12-wave variant where it is not instantiated, must not
  // silently launch another kernel under the requested name
  // variants: 0 / 1 (G8A) / 2 (12 waves); + 4: the 3-slot chunk ring (blocks with NS <= 10)
  // + 8: lattice spans (blocks 14-16: Cin 160, dilation 2), variants 0 / 1 / 4
  if (!(p.npi == 0 || p.npi == 1 || p.npi == 2 || p.npi == 4 || p.npi == 6 || p.npi == 8 || p.npi == 9 ||
        p.npi == 10 || p.npi == 12))
    throw std::invalid_argument("fused_ir_stream: variant must be 0, 1, 2, 4, 6 (+ 8 for lattice: 8, 9, 10, 12)");
  if (lat) {
    // window pitch 17 + 3 at W = 33; 3 halo rounds per expansion wave (<= 192 px)
    if (KS == 5 && NS == 10) {
      if (p.npi == 9) launch_stream<5, 10, 3, 1, 20, 9>(a, st);
      else if (p.npi == 10) launch_stream<5, 10, 3, 1, 20, 10>(a, st);
      else if (p.npi == 12) launch_stream<5, 10, 3, 1, 20, 12>(a, st);
      else launch_stream<5, 10, 3, 1, 20, 8>(a, st);
      return;
    }
    if (KS == 5 && NS == 20 && p.npi == 9) {
      launch_stream<5, 20, 3, 1, 20, 9>(a, st);
      return;
    }
    throw std::invalid_argument("fused_ir_stream: lattice instantiations: 160->160 (8, 9, 10, 12), 160->320 (9)");
  }
  if ((p.npi & 3) == 2 && (p.dil != 1 || NS > 6))
    throw std::invalid_argument("fused_ir_stream: the 12-wave variant needs dilation 1 and Cout <= 96");
  if ((p.npi & 4) && NS > 10)
    throw std::invalid_argument("fused_ir_stream: the 3-slot variant is for Cout <= 160 (wider blocks use 3 slots)");
  // 12-wave variant: blocks 7-12 (Cout <= 96; at Cout 160 the accumulators spill at 168 VGPRs
  // even with the register-lean depthwise -- block 13: 8 spills; the lattice form of blocks
  // 14-15 fits, its expansion waves hold 3 halo rounds instead of 4-5)
#define STREAM12(K_, N_) ((N_) <= 6 ? 2 : 0)
#define STREAM(K_, N_)                                   \
  if (KS == K_ && NS == N_) {                            \
    if (p.dil == 1 && p.npi == 2) launch_stream<K_, N_, 4, 1, 49, STREAM12(K_, N_)>(a, st);  \
    else if (p.dil == 1 && p.npi == 6) launch_stream<K_, N_, 4, 1, 49, 4 + STREAM12(K_, N_)>(a, st);  \
    else if (p.dil == 1 && p.npi == 1) launch_stream<K_, N_, 4, 1, 49, 1>(a, st);        \
    else if (p.dil == 1 && p.npi == 4) launch_stream<K_, N_, 4, 1, 49, 4>(a, st);        \
    else if (p.dil == 1) launch_stream<K_, N_, 4, 1, 49, 0>(a, st);                      \
    else if (p.npi == 1) launch_stream<K_, N_, 5, 2, 49, 1>(a, st);                      \
    else if (p.npi == 4) launch_stream<K_, N_, 5, 2, 49, 4>(a, st);                      \
    else launch_stream<K_, N_, 5, 2, 49, 0>(a, st);                                      \
    return;                                              \
  }
  // blocks 7-9 (64->64), 10 (64->96), 11-12 (96->96), 13 (96->160), 14-15 (160->160)
  STREAM(2, 4) STREAM(2, 6) STREAM(3, 6) STREAM(3, 10) STREAM(5, 10)
  // block 16 (160->320, dilation 2): group 8 on the expansion waves only (the projection
  // waves' accumulators for 2.5 groups x 20 subtiles would not fit 256 VGPRs)
  if (KS == 5 && NS == 20 && p.dil == 2) {
    launch_stream<5, 20, 5, 2, 49, 1>(a, st);
    return;
  }
#undef STREAM
#undef STREAM12
  throw std::invalid_argument("fused_ir_stream: no instantiation for this (Cin, Cout)");
}

// out = act(sum_h part[h] + bias (+ residual)), bf16: the combine of the hidden-split stream
// and of the split-K grouped ASPP GEMM (fixed summation order h = 0..HS-1, so the result is
// a function of the inputs alone)
// HSM: compile-time bound on HS, so every slab's loads (and the residual's) are issued before
// the first add -- one L2 round trip per unit instead of HS dependent ones (the runtime-HS loop
// ran 4.5-5 us per combine at batch 1, profiles/r6b_b1_layer_times.txt)
template <int HSM>
__global__ __launch_bounds__(256) void stream_combine_kernel(const float* __restrict__ part, const float* __restrict__ bp,
                                                             const bf16* __restrict__ res, bf16* __restrict__ out,
                                                             int HS, long long M, int Cout, int relu) {
  const long long units = M * (Cout / 8);
  const long long slab = M * Cout;
  const int cg = Cout / 8;
  for (long long u = blockIdx.x * 256ll + threadIdx.x; u < units; u += (long long)gridDim.x * 256) {
    const long long m = units < (1ll << 31) ? (long long)((int)u / cg) : u / cg;
    const int c = (int)(u - m * cg) * 8;
    const float* q = part + m * Cout + c;
    f32x4 s0 = *reinterpret_cast<const f32x4*>(bp + c), s1 = *reinterpret_cast<const f32x4*>(bp + c + 4);
    bf16x8 r = zero8();
    if constexpr (HSM > 0) {
      f32x4 p0[HSM], p1[HSM];
#pragma unroll
      for (int h = 0; h < HSM; ++h) {
        if (h < HS) {
          p0[h] = *reinterpret_cast<const f32x4*>(q + h * slab);
          p1[h] = *reinterpret_cast<const f32x4*>(q + h * slab + 4);
        }
      }
      if (res) r = ld8(res + m * Cout + c);
#pragma unroll
      for (int h = 0; h < HSM; ++h) {  // fixed order h = 0..HS-1
        if (h < HS) {
          s0 += p0[h];
          s1 += p1[h];
        }
      }
    } else {  // HS > 8 (hidden splits up to the chunk count): the runtime loop
      for (int h = 0; h < HS; ++h) {
        s0 += *reinterpret_cast<const f32x4*>(q + h * slab);
        s1 += *reinterpret_cast<const f32x4*>(q + h * slab + 4);
      }
      if (res) r = ld8(res + m * Cout + c);
    }
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = s0[e] + (float)r[e];
      v[e + 4] = s1[e] + (float)r[e + 4];
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)(relu ? fmaxf(v[e], 0.f) : v[e]);
    st8(out + m * Cout + c, o);
  }
}

void stream_combine(const float* part, const float* bp, const bf16* res, bf16* out, int HS, long long M, int Cout,
                    hipStream_t st, int act) {
  if (act != 0 && act != 1) throw std::invalid_argument("stream_combine: act 0 (none) or 1 (relu)");
  if (Cout % 8 || HS < 1 || M < 1) throw std::invalid_argument("stream_combine: Cout % 8, HS >= 1");
  const long long units = M * (Cout / 8);
  const int grid = (int)std::min<long long>((units + 255) / 256, 2048);
  if (HS <= 4)
    hipLaunchKernelGGL(stream_combine_kernel<4>, dim3(grid), dim3(256), 0, st, part, bp, res, out, HS, M, Cout, act);
  else if (HS <= 8)
    hipLaunchKernelGGL(stream_combine_kernel<8>, dim3(grid), dim3(256), 0, st, part, bp, res, out, HS, M, Cout, act);
  else
    hipLaunchKernelGGL(stream_combine_kernel<0>, dim3(grid), dim3(256), 0, st, part, bp, res, out, HS, M, Cout, act);
  check_launch("stream_combine");
}

}  // namespace ssa
