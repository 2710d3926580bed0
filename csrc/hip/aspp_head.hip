// DeepLabv3 head: ASPP projection (1x1, K = 4 x 256 concatenated branches -> 256,
// + bias + per-image pooling bias + ReLU) fused with the 1x1 logits conv
// (256 -> num_classes), gfx950.
//
//   proj[m, :]   = relu( Wp . cat[m, :] + bp + img_bias[m / HW] )       (bf16, on chip)
//   logits[m, :] = Wl . proj[m, :] + bl                                  (bf16, ldo stride)
//
// Round 1 ran this as a hipBLASLt GEMM + a bias/ReLU pass + a logits GEMM (31.4 + 7.5 +
// 14.8 us at B = 32, profiles/r1_hip_v10_layer_times.txt); the reference runs the whole
// network as one Edge TPU call (/root/reference/sem_seg_server.py:162).
//
// Work decomposition (MI355X-first):
//   * one 512-thread workgroup (8 waves, 2 per SIMD) per G pixel groups of 16
//     (G = 9 at B = 32: 2178 groups -> 242 workgroups, one per CU, 95 % of the chip);
//   * the projection's 256 output channels are split over the 8 waves (32 each), so
//     the pixel operand (the 2 KiB/pixel concat row, the bulk of the HBM traffic) is
//     fetched ONCE per workgroup and shared through LDS; each wave keeps its 32-channel
//     weight slice flowing global(L2) -> VGPRs two chunks ahead (MFMA A operand,
//     host-packed in fragment order: one lane-linear 16-byte load per fragment);
//   * the pixel tile streams through a 2-slot LDS ring in 64-channel chunks; staging
//     loads for chunk c+2 are issued at step c and written to LDS at the end of step
//     c+1 (two compute steps of latency cover), one barrier per step. Each thread's
//     staging piece is 16 bytes of one pixel row, 8 threads per 128-byte line, and the
//     LDS image is the MFMA B-fragment order with an XOR swizzle on the lane slot
//     (lane ^ (kq*2 + kk*8)) so both the staging ds_write_b128 (2 pixels x 8 octets per
//     16-lane group) and the lane-linear fragment ds_read_b128 are bank-conflict free;
//   * epilogue: bias + image bias + ReLU -> bf16 projection tile in LDS (pitch 528 B:
//     conflict-free 8-byte writes and 16-byte B-fragment reads), then the logits GEMM
//     (K = 256, 2 16-channel subtiles) straight from that tile. The projection never
//     touches HBM.
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

constexpr int kKC = 2;           // 32-deep k-steps per chunk (64 channels)
constexpr int kTP = 264;         // projection tile pitch (bf16 elements, 528 B)
constexpr int kNP = 256;         // projection channels

struct HeadArgs {
  const bf16* cat; const bf16* wp; const float* bp; const float* img_bias;
  const bf16* wl; const float* bl; bf16* out;
  int M, HW, ldo;
};

__device__ __forceinline__ int frag_slot(int lane, int kk) { return lane ^ (((lane >> 4) * 2 + kk * 8) & 15); }

// NWH = 16 (round 3): one projection subtile per wave, twice the waves per CU to cover the
// staging / LDS latency (the grouped ASPP GEMM gained 20 % from the same change)
template <int G, int KS, int NWH>
__global__ __launch_bounds__(NWH * 64) void aspp_head_kernel(HeadArgs a) {
  constexpr int kHW = NWH, kHT = NWH * 64;
  constexpr int NSUB = 16 / NWH;                  // projection subtiles per wave
  constexpr int NCH = KS / kKC;
  constexpr int SLOT = G * kKC * 1024;
  constexpr int NPC = G * 16 * 8;                 // 16-byte staging pieces per chunk
  constexpr int NLD = (NPC + kHT - 1) / kHT;
  constexpr int K = KS * 32;
  static_assert(KS % kKC == 0, "K must be a multiple of 64");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int row0 = blockIdx.x * G * 16;

  // ---- staging pieces of this thread: piece i = (pixel pl = i / 8, octet o = i % 8) of
  // a chunk's 128-byte row segment; octet o is k-step kk = o / 4, lane quarter kq = o % 4.
  // Branch-free: every thread issues NLD loads per chunk (pieces past the tile re-read
  // piece NPC-1 and land in a 16-byte sink), so the wait counts are exact on every path.
  constexpr int SINK = (2 * SLOT > G * 16 * kTP * 2 ? 2 * SLOT : G * 16 * kTP * 2);
  size_t goff[NLD];
  int loff[NLD];
#pragma unroll
  for (int q = 0; q < NLD; ++q) {
    const int i = min(tid + q * kHT, NPC - 1);
    const int pl = i >> 3, o = i & 7, kk = o >> 2, kqq = o & 3;
    const int m = min(row0 + pl, a.M - 1);  // tail rows re-read a valid row (outputs dropped)
    goff[q] = (size_t)m * K + o * 8;
    const int l = kqq * 16 + (pl & 15);
    loff[q] = tid + q * kHT < NPC ? ((pl >> 4) * kKC + kk) * 1024 + frag_slot(l, kk) * 16 : -1;
  }
  bf16x8 stg[2][NLD];
  auto stage_load = [&](int c, int s) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) stg[s][q] = ld8(a.cat + goff[q] + c * 64);
  };
  auto stage_store = [&](int s, int slot) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int off = loff[q] < 0 ? SINK : slot * SLOT + loff[q];
      *reinterpret_cast<bf16x8*>(smem + off) = stg[s][q];
    }
  };
  // ---- this wave's projection weights: subtiles n = NSUB*wid + {0 .. NSUB-1}, [n][k][lane][8]
  bf16x8 afr[3][kKC][NSUB];
  const bf16* wpw = a.wp + ((size_t)(NSUB * wid) * KS * 64 + lane) * 8;
  auto a_load = [&](int c, int s) {
#pragma unroll
    for (int kk = 0; kk < kKC; ++kk)
#pragma unroll
      for (int n = 0; n < NSUB; ++n) afr[s][kk][n] = ld8(wpw + ((size_t)n * KS + c * kKC + kk) * 512);
  };

  f32x4 acc[G][NSUB];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int n = 0; n < NSUB; ++n) acc[g][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage_load(0, 0);
  a_load(0, 0);
  if (NCH > 1) {
    stage_load(1, 1);
    a_load(1, 1);
  }
  stage_store(0, 0);
  __syncthreads();

#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    // chunk c+2's loads go out first (staging set c&1 was written to LDS at step c-1)
    if (c + 2 < NCH) {
      stage_load(c + 2, c & 1);
      a_load(c + 2, (c + 2) % 3);
    }
    __builtin_amdgcn_sched_barrier(0);
    const char* sl = smem + (c & 1) * SLOT;
#pragma unroll
    for (int kk = 0; kk < kKC; ++kk) {
      const int fs = frag_slot(lane, kk) * 16;
      bf16x8 b[G];  // all G fragment reads in flight, then the 2G MFMAs
#pragma unroll
      for (int g = 0; g < G; ++g) b[g] = *reinterpret_cast<const bf16x8*>(sl + (g * kKC + kk) * 1024 + fs);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int n = 0; n < NSUB; ++n)
          acc[g][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[c % 3][kk][n], b[g], acc[g][n], 0, 0, 0);
    }
    // slot (c+1)&1 was last read at step c-1 (behind that step's barrier)
    if (c + 1 < NCH) stage_store((c + 1) & 1, (c + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue 1: projection bias + image bias + ReLU -> bf16 tile in LDS
  bf16* T = reinterpret_cast<bf16*>(smem);
#pragma unroll
  for (int n = 0; n < NSUB; ++n) {
    const int ch = (NSUB * wid + n) * 16 + kq * 4;
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(a.bp + ch);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int m = min(row0 + g * 16 + r16, a.M - 1);
      f32x4 v = acc[g][n] + b4;
      if (a.img_bias) v += *reinterpret_cast<const f32x4*>(a.img_bias + (size_t)(m / a.HW) * kNP + ch);
      const bf16x4 o = {(bf16)fmaxf(v[0], 0.f), (bf16)fmaxf(v[1], 0.f), (bf16)fmaxf(v[2], 0.f),
                        (bf16)fmaxf(v[3], 0.f)};
      *reinterpret_cast<bf16x4*>(T + (g * 16 + r16) * kTP + ch) = o;
    }
  }
  __syncthreads();

  // ---- epilogue 2: logits = Wl . proj + bl (two 16-class subtiles, K = 256)
  const f32x4 bl0 = *reinterpret_cast<const f32x4*>(a.bl + kq * 4);
  const f32x4 bl1 = *reinterpret_cast<const f32x4*>(a.bl + 16 + kq * 4);
  for (int g = wid; g < G; g += kHW) {
    f32x4 l0 = bl0, l1 = bl1;
#pragma unroll
    for (int k = 0; k < kNP / 32; ++k) {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(T + (g * 16 + r16) * kTP + k * 32 + kq * 8);
      const bf16x8 w0 = ld8(a.wl + ((size_t)k * 64 + lane) * 8);
      const bf16x8 w1 = ld8(a.wl + ((size_t)(kNP / 32 + k) * 64 + lane) * 8);
      l0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, b, l0, 0, 0, 0);
      l1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, b, l1, 0, 0, 0);
    }
    const int m = row0 + g * 16 + r16;
    if (m < a.M) {
      bf16* dst = a.out + (size_t)m * a.ldo;
      const bf16x4 o0 = {(bf16)l0[0], (bf16)l0[1], (bf16)l0[2], (bf16)l0[3]};
      const bf16x4 o1 = {(bf16)l1[0], (bf16)l1[1], (bf16)l1[2], (bf16)l1[3]};
      if (kq * 4 < a.ldo) *reinterpret_cast<bf16x4*>(dst + kq * 4) = o0;
      if (16 + kq * 4 < a.ldo) *reinterpret_cast<bf16x4*>(dst + 16 + kq * 4) = o1;
    }
  }
}

template <int G, int KS, int NWH>
void launch_head(const HeadArgs& a, hipStream_t s) {
  const size_t lds = aspp_head_lds(G, KS * 32);
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&aspp_head_kernel<G, KS, NWH>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "aspp_head attr");
    attr = true;
  }
  const int grid = cdiv(a.M, G * 16);
  hipLaunchKernelGGL((aspp_head_kernel<G, KS, NWH>), dim3(grid), dim3(NWH * 64), lds, s, a);
  check_launch("aspp_head");
}

}  // namespace

size_t aspp_head_lds(int G, int K) {
  const size_t ring = (size_t)2 * G * kKC * 1024, tile = (size_t)G * 16 * kTP * 2;
  (void)K;
  return (ring > tile ? ring : tile) + 16;  // + the staging sink
}

void aspp_head(const AsppHeadParams& p, hipStream_t s) {
  if (p.K % 64 || p.N != kNP || p.ncls < 1 || p.ncls > 32 || p.ldo % 4 || p.ldo < p.ncls || p.ldo > 32)
    throw std::invalid_argument("aspp_head: K % 64, N == 256, ncls <= 32, ldo % 4 in [ncls, 32]");
  if (p.M <= 0 || (p.img_bias && p.HW <= 0)) throw std::invalid_argument("aspp_head: bad M / HW");
  if ((long long)p.M * p.K >= (1LL << 40)) throw std::invalid_argument("aspp_head: input too large");
  HeadArgs a{p.cat, p.wp, p.bp, p.img_bias, p.wl, p.bl, p.out, p.M, p.HW > 0 ? p.HW : 1, p.ldo};
  const int KS = p.K / 32;
#define HEAD(G_, KS_)                                              \
  if (p.G == G_ && KS == KS_) {                                    \
    if (p.waves == 16) launch_head<G_, KS_, 16>(a, s);             \
    else launch_head<G_, KS_, 8>(a, s);                            \
    return;                                                        \
  }
  HEAD(1, 32) HEAD(2, 32) HEAD(3, 32) HEAD(5, 32) HEAD(9, 32)
#undef HEAD
  throw std::invalid_argument("aspp_head: no instantiation for this (G, K)");
}

}  // namespace ssa
