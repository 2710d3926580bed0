// Dilated KxK stride-1 convolution (the ASPP atrous branches) as a tap loop over
// weight-streamed MFMA GEMMs, NHWC bf16 -- pw_conv.hip's structure extended to taps:
//
//   out[p, co_off + n] = act( bias[n] + sum_t sum_c W[n][t][c] * in[p + d_t][c] )
//
// The LDS-DMA implicit GEMM (conv_gemm.hip, conv_glds_kernel) gathers a 128-row
// im2col tile of BOTH operands through LDS every 64-deep K step: ~8 DMA
// instructions with per-row bounds checks per wave per step, a barrier per step,
// and it tops out near 450 TF/s on the 33x33 ASPP shapes whatever its ring depth.
// Here, per tap:
//   * pixel operand (MFMA B): each of the 8 waves gathers ITS 32 pixels' Cin row
//     at the tap offset straight into VGPRs (16 B per lane per 32-deep step, zero
//     outside the image) -- no LDS, no im2col image; the next tap's rows are
//     prefetched into a second register set while this tap's MFMAs run;
//   * weight operand (MFMA A): the tap's [128 out-ch x Cin] slice, host-packed in
//     MFMA fragment order, is ONE contiguous LDS-DMA copy (double-buffered across
//     taps), read back as conflict-free contiguous ds_read_b128;
//   * the 256 pixel x 128 channel accumulator stays in registers across all taps;
//     one epilogue (bias, act, permlane16-widened 16-byte buffer stores).
// Taps are skipped per workgroup when all its pixels see padding; with the
// tap-validity row permutation (hip_ops.tap_group_perm) every workgroup is
// tap-uniform, so only live taps are computed (ASPP rates 6/12/18 on 33x33:
// 6.95 / 5.17 / 3.64 of 9 on average).
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

constexpr int kTapWaves = 8;   // 512 threads; 2 waves per SIMD
constexpr int kTapMT = 2;      // 32 pixels per wave -> 256-pixel tile
constexpr int kTapNS = 8;      // 8 x 16 = 128 output channels per workgroup

struct TapArgs {
  const bf16* in; const bf16* w; const float* bias; bf16* out; const int* perm;
  int B, H, W, Cin, Cout, KH, KW, dil, ldo, co_off, act, Mrows, ngroups, out_bytes;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int KS>
__global__ __launch_bounds__(64 * kTapWaves) void tap_conv_kernel(TapArgs a) {
  constexpr int MT = kTapMT, NS = kTapNS;
  constexpr int TAP_B = NS * KS * 1024;  // one tap's weight slice for this workgroup
  constexpr int NDMA = TAP_B / 1024 / kTapWaves;  // 1 KiB DMA wave-instructions per wave
  static_assert(NDMA * 1024 * kTapWaves == TAP_B, "tap slice must split over the waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // tap-mask reduction word: the start of LDS buffer 1, which no DMA writes before
  // the first in-loop barrier (KS = 10 uses all 160 KiB for the two buffers)
  int& s_tap = *reinterpret_cast<int*>(smem + TAP_B);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int tiles_m = cdiv_dev(a.Mrows, 16 * MT * kTapWaves);
  const int bid = xcd_remap(blockIdx.x, tiles_m * a.ngroups);
  const int tm = bid / a.ngroups, g = bid - tm * a.ngroups;
  const int HW = a.H * a.W;
  const int taps = a.KH * a.KW;

  // this lane's pixels (B-fragment column r16 of each 16-pixel group)
  int pb[MT], py[MT], px[MT];
  bool pv[MT];
  int tapbits = 0;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = tm * 16 * MT * kTapWaves + wid * 16 * MT + i * 16 + r16;
    const int p = row < a.Mrows ? (a.perm ? a.perm[row] : row) : -1;
    pv[i] = p >= 0;
    const int pp = pv[i] ? p : 0;
    pb[i] = pp / HW;
    const int rem = pp - pb[i] * HW;
    py[i] = rem / a.W;
    px[i] = rem - py[i] * a.W;
    if (pv[i])
      for (int t = 0; t < taps; ++t) {
        const int iy = py[i] + (t / a.KW - a.KH / 2) * a.dil, ix = px[i] + (t % a.KW - a.KW / 2) * a.dil;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) tapbits |= 1 << t;
      }
  }
  if (tid == 0) s_tap = 0;
  __syncthreads();
  if (tapbits) atomicOr(&s_tap, tapbits);
  __syncthreads();
  const int tapmask = __builtin_amdgcn_readfirstlane(s_tap);

  // weight slice of tap t for channel group g: packed [tap][group][NS][KS][64][8]
  auto issue = [&](int t, int buf) {
    const char* src = reinterpret_cast<const char*>(a.w) + ((size_t)t * a.ngroups + g) * TAP_B +
                      wid * 1024 + lane * 16;
    char* dst = smem + buf * TAP_B + wid * 1024;
#pragma unroll
    for (int q = 0; q < NDMA; ++q)
      __builtin_amdgcn_global_load_lds(src + q * kTapWaves * 1024,
                                       (lds_ptr_t)(dst + q * kTapWaves * 1024), 16, 0, 0);
  };
  auto load_px = [&](int t, bf16x8 (&fr)[KS][MT]) {
    const int dy = (t / a.KW - a.KH / 2) * a.dil, dx = (t % a.KW - a.KW / 2) * a.dil;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int iy = py[i] + dy, ix = px[i] + dx;
      const bool ok = pv[i] && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const bf16* src = a.in + ((size_t)(pb[i] * a.H + (ok ? iy : 0)) * a.W + (ok ? ix : 0)) * a.Cin + kq * 8;
#pragma unroll
      for (int k = 0; k < KS; ++k)
        fr[k][i] = (ok && k * 32 + kq * 8 < a.Cin) ? ld8(src + k * 32) : zero8();
    }
  };

  f32x4 acc[MT][NS];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf, const bf16x8 (&fr)[KS][MT]) {
    const char* Wl = smem + buf * TAP_B + lane * 16;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(Wl + (j * KS + k) * 1024);
#pragma unroll
        for (int i = 0; i < MT; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, fr[k][i], acc[i][j], 0, 0, 0);
      }
    }
  };

  // live taps walked as set bits of the (wave-uniform) mask; two register sets for
  // the pixel rows so that every array index is static
  bf16x8 f0[KS][MT], f1[KS][MT];
  int rem = tapmask;
  if (rem) {
    issue(__builtin_ctz(rem), 0);
    load_px(__builtin_ctz(rem), f0);
  }
  // step s: wait for tap s (DMA + rows), barrier (everyone is past tap s-1, so the
  // other LDS buffer is free), prefetch tap s+1, compute tap s
  int s = 0;
  auto step = [&](const bf16x8 (&cur)[KS][MT], bf16x8 (&nxt)[KS][MT]) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    rem &= rem - 1;  // drop the tap being computed
    if (rem) {
      issue(__builtin_ctz(rem), (s + 1) & 1);
      load_px(__builtin_ctz(rem), nxt);
    }
    compute(s & 1, cur);
    ++s;
  };
  while (rem) {
    step(f0, f1);
    if (!rem) break;
    step(f1, f0);
  }

  // epilogue: pair subtiles (2p, 2p+1) -> 8 consecutive channels per lane
  const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_bytes, 0x00020000);
  const float lo = a.act == ACT_NONE ? -INFINITY : 0.f;
  const float hi = a.act == ACT_RELU6 ? 6.f : INFINITY;
#pragma unroll
  for (int p = 0; p < NS / 2; ++p) {
    const int n = g * NS * 16 + (2 * p + (kq & 1)) * 16 + (kq >> 1) * 8;
    const bool nv = n < a.Cout;
    float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
    if (nv) {
      b0 = *reinterpret_cast<const float4*>(a.bias + n);
      b1 = *reinterpret_cast<const float4*>(a.bias + n + 4);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * p][q]),
                                                        __float_as_uint(acc[i][2 * p + 1][q]), false, false);
        v[q] = __uint_as_float(r[0]);
        v[q + 4] = __uint_as_float(r[1]);
      }
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
      bf16x8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (bf16)fminf(fmaxf(v[q], lo), hi);
      const int pix = (pb[i] * a.H + py[i]) * a.W + px[i];
      const int off = (nv && pv[i]) ? (pix * a.ldo + a.co_off + n) * 2 : a.out_bytes;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), orsrc, off, 0, 0);
    }
  }
}

template <int KS>
void launch_tap(const TapArgs& a, hipStream_t s) {
  constexpr size_t lds = 2 * (size_t)kTapNS * KS * 1024;
  static bool attr_set = false;
  if (!attr_set) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&tap_conv_kernel<KS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "tap_conv attr");
    attr_set = true;
  }
  const int grid = cdiv(a.Mrows, 16 * kTapMT * kTapWaves) * a.ngroups;
  hipLaunchKernelGGL((tap_conv_kernel<KS>), dim3(grid), dim3(64 * kTapWaves), lds, s, a);
  check_launch("tap_conv");
}

}  // namespace

void tap_conv(const TapConvParams& p, hipStream_t s) {
  const int KS = (p.Cin + 31) / 32;
  if (p.Cin % 8 || p.Cout % 8 || p.ldo % 8 || p.co_off % 8 || p.co_off + p.Cout > p.ldo)
    throw std::invalid_argument("tap_conv: Cin, Cout, ldo, co_off must be multiples of 8");
  if (p.KH * p.KW > 16 || p.KH % 2 == 0 || p.KW % 2 == 0) throw std::invalid_argument("tap_conv: bad kernel size");
  const long long out_bytes = (long long)p.B * p.H * p.W * p.ldo * 2;
  if (out_bytes >= (1LL << 31) || (long long)p.B * p.H * p.W * p.Cin >= (1LL << 31))
    throw std::invalid_argument("tap_conv: tensor too large for 32-bit offsets");
  TapArgs a{p.in, p.w, p.bias, p.out, p.perm, p.B, p.H, p.W, p.Cin, p.Cout, p.KH, p.KW, p.dil,
            p.ldo, p.co_off, p.act, p.perm ? p.Mp : p.B * p.H * p.W,
            (p.Cout + 16 * kTapNS - 1) / (16 * kTapNS), (int)out_bytes};
  switch (KS) {
    case 2: launch_tap<2>(a, s); break;
    case 4: launch_tap<4>(a, s); break;
    case 5: launch_tap<5>(a, s); break;
    case 8: launch_tap<8>(a, s); break;
    case 10: launch_tap<10>(a, s); break;
    default: throw std::invalid_argument("tap_conv: Cin has no instantiation (need 64/128/160/256/320)");
  }
}

int tap_conv_group_channels() { return 16 * kTapNS; }

}  // namespace ssa
