// Pointwise (1x1, stride 1) convolution as a weight-streamed MFMA GEMM, NHWC bf16.
//
//   out[m, co_off + n] = act( sum_k W[n][k] * in[m][k] + bias[n] + img_bias[b(m)][n] + res[m][n] )
//
// Built for the shapes that dominate DeepLabv3-MobileNetV2 at OS16: the 1x1
// expansions (K = Cin <= 320, N = 6*Cin), the ASPP 1x1 branch and the logits.
// The generic implicit-GEMM kernels (conv_gemm.hip) give every wave its own
// fragments of BOTH operands, so each weight byte is fetched from L2 once per
// wave and every 64-pixel tile re-streams the whole weight slice: ~520 MB of
// L2->CU traffic for one 160->960 expansion over 32 frames of 33x33.
//
// Here the roles are split by reuse:
//   * pixel operand (MFMA B): a wave owns 16*MT pixels and keeps ALL of their K
//     in VGPRs for the whole kernel (one 16-byte load per lane per 32-deep K step);
//   * weight operand (MFMA A): streamed through LDS in 64-output-channel chunks,
//     double-buffered with gfx950 LDS-DMA (global_load_lds_dwordx4: no VGPR
//     staging, no ds_write pass). The host pre-packs W in MFMA fragment order
//     ([chunk][subtile j][k-step][lane][8]), so one DMA wave-instruction is a
//     contiguous 1 KiB copy and every ds_read_b128 of a fragment reads 1 KiB
//     contiguous LDS: bank-conflict free with no swizzle arithmetic at all;
//   * a workgroup walks `nch` consecutive chunks for its pixel tile, so the
//     pixel loads are amortised over 64*nch output channels.
// Epilogue: with A = weights the 16x16x32 C fragment gives a lane 4 consecutive
// channels of one pixel (8-byte stores). One v_permlane16_swap per accumulator
// dword pairs neighbouring 16-channel subtiles so that each lane ends up with 8
// consecutive channels: half as many store instructions, 16 bytes each, and the
// bias / residual loads become 16-byte vectors too.
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

struct PwArgs {
  const bf16* in; const bf16* w; const float* img_bias; const bf16* res;
  bf16* out;
  int M, K, N, HW, ldo, co_off, ldr, act, nch, ngroups, NC, out_bytes, out_f16;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int MT, int KS>
__global__ __launch_bounds__(256) void pw_conv_kernel(PwArgs a) {
  // one 64-channel chunk: 4 subtiles x KS steps x 1 KiB of weights, then 1 KiB holding
  // the chunk's 64 fp32 biases (the epilogue reads them from LDS: a global load issued
  // after the next chunk's DMA would make the compiler drain that DMA with vmcnt(0))
  constexpr int CHUNK_B = (4 * KS + 1) * 1024;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int tiles_m = cdiv_dev(a.M, 64 * MT);
  // consecutive logical blocks (one XCD under round-robin dispatch) share a pixel tile
  const int bid = xcd_remap(blockIdx.x, tiles_m * a.ngroups);
  const int tm = bid / a.ngroups, g = bid - tm * a.ngroups;
  const int c_begin = g * a.nch;
  const int c_end = min(c_begin + a.nch, a.NC);
  const int pix0 = tm * 64 * MT + wid * 16 * MT;

  auto issue = [&](int c, int buf) {
    const char* src = reinterpret_cast<const char*>(a.w) + (size_t)c * CHUNK_B + wid * 1024 + lane * 16;
    char* dst = smem + buf * CHUNK_B + wid * 1024;
#pragma unroll
    for (int q = 0; q < KS; ++q)
      __builtin_amdgcn_global_load_lds(src + q * 4096, (lds_ptr_t)(dst + q * 4096), 16, 0, 0);
    if (wid == 0)
      __builtin_amdgcn_global_load_lds(src + KS * 4096, (lds_ptr_t)(dst + KS * 4096), 16, 0, 0);
  };
  issue(c_begin, 0);  // in flight under the pixel loads

  bf16x8 bfr[KS][MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = pix0 + i * 16 + r16;
    const bool mv = m < a.M;
    const bf16* src = a.in + (size_t)(mv ? m : 0) * a.K + kq * 8;
#pragma unroll
    for (int k = 0; k < KS; ++k)
      bfr[k][i] = (mv && k * 32 + kq * 8 < a.K) ? ld8(src + k * 32) : zero8();
  }

  // Output through a range-checked buffer descriptor: a store whose offset lies
  // beyond num_records is dropped by the hardware, so masked lanes (M tail,
  // channel padding) need no branch.
  const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_bytes, 0x00020000);
  // activation as a branch-free clamp
  const float lo = a.act == ACT_NONE ? -INFINITY : 0.f;
  const float hi = a.act == ACT_RELU6 ? 6.f : INFINITY;

  for (int c = c_begin, it = 0; c < c_end; ++c, ++it) {
    // chunk c has landed (this wave's DMA + everyone's, via the barrier), and every
    // wave is done reading the other buffer (chunk c-1): refill it with chunk c+1.
    // VMEM ops younger than chunk c's DMA: only the previous chunk's 2*MT stores.
    // vmcnt(0): the chunk's LDS-DMA must have landed. A counted wait that left the previous
    // chunk's 2*MT stores in flight (vmcnt(2*MT)) assumed the stores retire after the older
    // DMA; under memory pressure from concurrent kernels they can retire first, the count
    // then passes with DMA pieces still in flight and the MFMAs read stale weights
    // (label maps differed in ~7 % of runs with plan copies on three streams,
    // scripts/debug_race.py).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // raw s_barrier: __syncthreads() carries a workgroup release that makes the
    // compiler drain every outstanding store (vmcnt(0)) first. LDS reads of the
    // previous chunk are all consumed by MFMAs already, so none is pending here.
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // this chunk's bias: LDS -> registers through inline-asm ds_reads. A compiler-
    // visible LDS read here gets a conservative vmcnt(0) in front of it (the
    // waitcnt pass cannot tell it apart from the in-flight LDS-DMA), which would
    // drain the previous chunk's stores; the wait above already covers the DMA.
    f32x4 bias4[2][2];
    {
      const unsigned bl = (unsigned)(uintptr_t)(lds_ptr_t)(smem + (it & 1) * CHUNK_B + 4 * KS * 1024) +
                          (((kq & 1) * 16 + (kq >> 1) * 8) << 2);
      asm volatile(
          "ds_read_b128 %0, %4\n\t"
          "ds_read_b128 %1, %4 offset:16\n\t"
          "ds_read_b128 %2, %4 offset:128\n\t"
          "ds_read_b128 %3, %4 offset:144\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=v"(bias4[0][0]), "=v"(bias4[0][1]), "=v"(bias4[1][0]), "=v"(bias4[1][1])
          : "v"(bl)
          : "memory");
    }
    if (c + 1 < c_end) issue(c + 1, (it + 1) & 1);
    const char* Wl = smem + (it & 1) * CHUNK_B + lane * 16;

    f32x4 acc[MT][4];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      bf16x8 afr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) afr[j] = *reinterpret_cast<const bf16x8*>(Wl + (j * KS + k) * 1024);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[j], bfr[k][i], acc[i][j], 0, 0, 0);
    }

    // epilogue: pair subtiles (2p, 2p+1) so every lane owns 8 consecutive channels
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = c * 64 + (2 * p + (kq & 1)) * 16 + (kq >> 1) * 8;
      const bool nv = n < a.N;
      const f32x4 b0 = bias4[p][0], b1 = bias4[p][1];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * p][q]),
                                                          __float_as_uint(acc[i][2 * p + 1][q]),
                                                          false, false);
          v[q] = __uint_as_float(r[0]);
          v[q + 4] = __uint_as_float(r[1]);
        }
        const int m = pix0 + i * 16 + r16;
        const bool ok = nv && m < a.M;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] += b0[q];
          v[q + 4] += b1[q];
        }
        if (a.img_bias && ok) {
          const float* ib = a.img_bias + (size_t)(m / a.HW) * a.N + n;
          const float4 i0 = *reinterpret_cast<const float4*>(ib);
          const float4 i1 = *reinterpret_cast<const float4*>(ib + 4);
          v[0] += i0.x; v[1] += i0.y; v[2] += i0.z; v[3] += i0.w;
          v[4] += i1.x; v[5] += i1.y; v[6] += i1.z; v[7] += i1.w;
        }
        if (a.res && ok) {
          const bf16x8 rv = ld8(a.res + (size_t)m * a.ldr + n);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] += (float)rv[q];
        }
        u32x4 ob;
        if (a.out_f16) {  // fp16 activations for the fp16 depthwise consumers (dw_proj.hip)
          f16x8 o;
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (_Float16)fminf(fmaxf(v[q], lo), hi);
          ob = __builtin_bit_cast(u32x4, o);
        } else {
          bf16x8 o;
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (bf16)fminf(fmaxf(v[q], lo), hi);
          ob = __builtin_bit_cast(u32x4, o);
        }
        const int off = ok ? (m * a.ldo + a.co_off + n) * 2 : a.out_bytes;  // >= num_records: dropped
        __builtin_amdgcn_raw_buffer_store_b128(ob, orsrc, off, 0, 0);
      }
    }
  }
}

template <int MT, int KS>
void launch_pw(const PwArgs& a, hipStream_t s) {
  constexpr size_t lds = 2 * (4 * KS + 1) * 1024;
  static bool attr_set = false;
  if (!attr_set) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&pw_conv_kernel<MT, KS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "pw_conv attr");
    attr_set = true;
  }
  const int grid = cdiv(a.M, 64 * MT) * a.ngroups;
  hipLaunchKernelGGL((pw_conv_kernel<MT, KS>), dim3(grid), dim3(256), lds, s, a);
  check_launch("pw_conv");
}

template <int MT>
bool dispatch_pw(const PwArgs& a, int KS, hipStream_t s) {
  switch (KS) {
    case 1: launch_pw<MT, 1>(a, s); return true;
    case 2: launch_pw<MT, 2>(a, s); return true;
    case 3: launch_pw<MT, 3>(a, s); return true;
    case 4: launch_pw<MT, 4>(a, s); return true;
    case 5: launch_pw<MT, 5>(a, s); return true;
    case 8: launch_pw<MT, 8>(a, s); return true;
    case 10: launch_pw<MT, 10>(a, s); return true;
    default: return false;
  }
}

}  // namespace

int pw_conv_supported_ks(int K) {
  const int ks = (K + 31) / 32;
  return (K % 8 == 0 && (ks <= 5 || ks == 8 || ks == 10)) ? ks : 0;
}

void pw_conv(const PwConvParams& p, hipStream_t s) {
  const int KS = pw_conv_supported_ks(p.K);
  if (!KS) throw std::invalid_argument("pw_conv: unsupported K");
  if (p.N % 8 || p.ldo % 8 || p.co_off % 8 || (p.res && p.ldr % 8))
    throw std::invalid_argument("pw_conv: N, ldo, co_off, ldr must be multiples of 8");
  if (p.nch < 1 || p.M <= 0) throw std::invalid_argument("pw_conv: bad nch / M");
  const long long out_bytes = (long long)p.M * p.ldo * 2;
  if (out_bytes >= (1LL << 31) || (long long)p.M * p.K >= (1LL << 31))
    throw std::invalid_argument("pw_conv: tensor too large for 32-bit buffer offsets");
  const int NC = (p.N + 63) / 64;
  PwArgs a{p.in, p.w, p.img_bias, p.res, p.out, p.M, p.K, p.N, p.HW, p.ldo, p.co_off,
           p.ldr, p.act, p.nch, (NC + p.nch - 1) / p.nch, NC, (int)out_bytes, p.out_f16};
  const bool ok = p.mt == 4 ? dispatch_pw<4>(a, KS, s) : dispatch_pw<2>(a, KS, s);
  if (!ok) throw std::invalid_argument("pw_conv: no kernel for this K");
}

}  // namespace ssa
