// Depthwise 3x3 (+bias, ReLU6) fused with the 1x1 projection (+bias, +residual)
// for the 33x33 MobileNetV2 blocks (hid 384..960, dilation 1 or 2), gfx950.
//
//   out[p, n] = bp[n] + res[p, n] + sum_c Wp[n][c] * relu6( bd[c] + sum_t wd[t][c] * h[p + d_t][c] )
//
// The unfused path writes the depthwise output (= the projection's whole K
// operand, 67 MB per 32 frames at hid 960) and reads it back; here it never
// leaves the VGPRs. Per 32-channel hidden chunk, each lane computes the depthwise
// result for 8 channels of ONE pixel -- exactly its B fragment of the projection's
// v_mfma_f32_16x16x32_bf16 (lane l: pixel l&15, channels 8*(l>>4)..+7).
//   * hidden taps: 9 x 16-byte global loads per lane per chunk (the 9 neighbours
//     overlap between the pixels of a workgroup, so L1 serves most of them),
//     prefetched one chunk ahead into a second register set;
//   * fp16 internals as the fused tile kernels: the expansion writes relu6(x) in
//     fp16 (pw_conv out_f16), the depthwise is 4 v_pk_fma_f16 per tap and its
//     result feeds v_mfma_f32_16x16x32_f16 with no conversion (fp32 accumulate);
//   * weights: per chunk one contiguous host-packed image [NS projection
//     subtiles in MFMA fragment order (fp16) | 9x32 fp16 depthwise weights | 32
//     fp16 depthwise biases], double-buffered through LDS with LDS-DMA;
//   * epilogue as pw_conv: permlane16-paired subtiles, 16-byte bias / residual
//     loads and range-checked buffer stores.
// Every channel slice of the projection is computed by the same workgroup (the
// depthwise is computed once per pixel, unlike a Cout-split grid).
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct DPPArgs {
  const f16* h; const f16* w; const float* bp; const bf16* res; bf16* out;
  int B, IH, IW, hid, Cout, OH, OW, stride, dil, out_bytes;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));


template <int NS, int NW>
__global__ __launch_bounds__(64 * NW) void dw_proj_kernel(DPPArgs a) {
  constexpr int CHUNK_B = (NS + 1) * 1024;  // NS KiB projection fragments + 1 KiB depthwise
  constexpr int NDMA = NS + 1;              // 1 KiB DMA pieces per chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int M = a.B * a.OH * a.OW;
  const int tiles = cdiv_dev(M, 16 * NW);
  const int m = xcd_remap(blockIdx.x, tiles) * 16 * NW + wid * 16 + r16;
  const bool mv = m < M;
  const int mm = mv ? m : 0;
  const int b = mm / (a.OH * a.OW);
  const int rem = mm - b * a.OH * a.OW;
  const int oy = rem / a.OW, ox = rem - (rem / a.OW) * a.OW;

  // the 9 tap offsets of this lane's pixel (element index of channel 0; -1: padding)
  int toff[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int iy = oy * a.stride + (t / 3 - 1) * a.dil, ix = ox * a.stride + (t % 3 - 1) * a.dil;
    const bool ok = mv && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
    toff[t] = ok ? ((b * a.IH + iy) * a.IW + ix) * a.hid + kq * 8 : -1;
  }
  const int nchunks = a.hid / 32;

  auto issue = [&](int c, int buf) {
    const char* src = reinterpret_cast<const char*>(a.w) + (size_t)c * CHUNK_B + lane * 16;
    char* dst = smem + buf * CHUNK_B;
    for (int q = wid; q < NDMA; q += NW)
      __builtin_amdgcn_global_load_lds(src + q * 1024, (lds_ptr_t)(dst + q * 1024), 16, 0, 0);
  };
  const f16x8 h0 = {0, 0, 0, 0, 0, 0, 0, 0}, h6 = {6, 6, 6, 6, 6, 6, 6, 6};
  auto load_taps = [&](int c, f16x8 (&v)[9]) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
      v[t] = toff[t] >= 0 ? *reinterpret_cast<const f16x8*>(a.h + toff[t] + c * 32) : h0;
  };

  f32x4 acc[NS];
#pragma unroll
  for (int n = 0; n < NS; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf, const f16x8 (&v)[9]) {
    const char* W = smem + buf * CHUNK_B;
    // depthwise: packed fp16 on this lane's 8 channels
    const f16* wd = reinterpret_cast<const f16*>(W + NS * 1024);  // [9][32] then bias [32]
    f16x8 d = *reinterpret_cast<const f16x8*>(wd + 9 * 32 + kq * 8);
#pragma unroll
    for (int t = 0; t < 9; ++t) d = v[t] * *reinterpret_cast<const f16x8*>(wd + t * 32 + kq * 8) + d;
    d = __builtin_elementwise_min(__builtin_elementwise_max(d, h0), h6);
    const char* Wl = W + lane * 16;
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const f16x8 af = *reinterpret_cast<const f16x8*>(Wl + n * 1024);
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, d, acc[n], 0, 0, 0);
    }
  };

  f16x8 va[9], vb[9];
  issue(0, 0);
  load_taps(0, va);
  int c = 0;
  // step: chunk c landed (DMA + taps) -> barrier (everyone past chunk c-1: its
  // buffer is free) -> prefetch chunk c+1 -> compute chunk c
  auto step = [&](const f16x8 (&cur)[9], f16x8 (&nxt)[9]) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + 1 < nchunks) {
      issue(c + 1, (c + 1) & 1);
      load_taps(c + 1, nxt);
    }
    compute(c & 1, cur);
    ++c;
  };
  while (c < nchunks) {
    step(va, vb);
    if (c >= nchunks) break;
    step(vb, va);
  }

  // epilogue: pair subtiles (2p, 2p+1) -> 8 consecutive channels per lane
  const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_bytes, 0x00020000);
#pragma unroll
  for (int p = 0; p < NS / 2; ++p) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * p][q]),
                                                      __float_as_uint(acc[2 * p + 1][q]), false, false);
      v[q] = __uint_as_float(r[0]);
      v[q + 4] = __uint_as_float(r[1]);
    }
    const int n = (2 * p + (kq & 1)) * 16 + (kq >> 1) * 8;
    const bool ok = mv && n < a.Cout;
    if (ok) {
      const float4 b0 = *reinterpret_cast<const float4*>(a.bp + n);
      const float4 b1 = *reinterpret_cast<const float4*>(a.bp + n + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
      if (a.res) {
        const bf16x8 rv = ld8(a.res + (size_t)m * a.Cout + n);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += (float)rv[q];
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (bf16)v[q];
    const int off = ok ? (m * a.Cout + n) * 2 : a.out_bytes;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), orsrc, off, 0, 0);
  }
}

template <int NS, int NW>
void launch_dwp(const DPPArgs& a, hipStream_t s) {
  constexpr size_t lds = 2 * (size_t)(NS + 1) * 1024;
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&dw_proj_kernel<NS, NW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "dw_proj attr");
    attr = true;
  }
  const int M = a.B * a.OH * a.OW;
  hipLaunchKernelGGL((dw_proj_kernel<NS, NW>), dim3(cdiv(M, 16 * NW)), dim3(64 * NW), lds, s, a);
  check_launch("dw_proj");
}

template <int NW>
void dispatch_dwp(const DPPArgs& a, int ns, hipStream_t s) {
  switch (ns) {
    case 4: launch_dwp<4, NW>(a, s); break;    // Cout 64
    case 6: launch_dwp<6, NW>(a, s); break;    // Cout 96
    case 10: launch_dwp<10, NW>(a, s); break;  // Cout 160
    case 20: launch_dwp<20, NW>(a, s); break;  // Cout 320
    default: throw std::invalid_argument("dw_proj_fused: unsupported Cout");
  }
}

// ---------------------------------------------------------------------------
// Row-tile variant: the per-lane tap gathers above re-read every hidden element
// ~9x through L1 (measured: slower than the unfused depthwise + GEMM pair). Here a
// workgroup owns TY full output rows of one image (stride 1), one wave per 16
// output pixels, and per 32-channel hidden chunk the (TY + 2*dil) x (OW + 2*dil)
// halo of the fp16 hidden tensor is copied ONCE into LDS by LDS-DMA (out-of-image
// pixels read a zero page), next to that chunk's weight image. The depthwise then
// reads its 9 taps from LDS.
__device__ __attribute__((aligned(16))) int4 g_dwp_zero[8];

// ST-stage LDS ring (ST - 1 chunks in flight across each barrier, counted vmcnt):
// per chunk a workgroup only has ~NS MFMAs per wave of work against a full L2/MALL
// round trip for the next chunk's halo, so one chunk of lookahead leaves the
// waves waiting on the DMA. XCD: row tiles of one image go to one XCD (their halo
// rows overlap, so the re-reads hit that XCD's L2).
template <int NS, int ST>
__global__ __launch_bounds__(1024) void dw_proj_rows_kernel(DPPArgs a, int TY, int HPP, int xcd) {
  // HPP: halo pixels rounded up to 64. The halo chunk is stored as 4 channel-octet
  // PLANES [octet][HPP pixels][16 B] (plane stride HPP * 16 B, a multiple of 1 KiB):
  // a depthwise ds_read_b128 lane group reads 16 distinct consecutive pixels of ONE
  // 16-byte bank slot column each, so it is conflict-free. Round 1 stored pixels as
  // 64-byte rows of all 4 octets: the 16 pixels of a lane group hit only 4 bank slots
  // (2-way conflicts on every depthwise read, ~1 conflict cycle per LDS instruction in
  // profiles/r1_hip_v10_pmc_summary.txt). One 1 KiB LDS-DMA piece = 64 pixels of one
  // octet plane (piece j: octet j % 4, pixels (j / 4) * 64 ..).
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int WB = (NS + 1) * 1024;            // weight image per chunk
  const int BUF = HPP * 64 + WB;             // halo [HPP][32 ch fp16] + weights
  const int NW = blockDim.x >> 6;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int dl = a.dil, HWW = a.OW + 2 * dl;  // halo row width
  const int rows_per_img = cdiv_dev(a.OH, TY);
  const int bid = xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int b = bid / rows_per_img, oy0 = (bid - b * rows_per_img) * TY;
  // this lane's output pixel
  const int p = wid * 16 + r16;
  const int py = p / a.OW, px = p - py * a.OW;
  const bool pv = p < TY * a.OW && oy0 + py < a.OH;
  const int PLANE = HPP * 16;
  const int dwbase = (pv ? (py * HWW + px) * 16 : 0) + kq * PLANE;  // halo byte offset of tap (0,0)
  const int m = (b * a.OH + oy0 + py) * a.OW + px;
  // DMA sources of this wave's halo pieces (element offsets for channel 0, -1: zero page)
  const int npieces = HPP / 16;
  constexpr int MAXP = 4;
  int hsrc[MAXP];
#pragma unroll
  for (int k = 0; k < MAXP; ++k) {
    const int piece = wid + k * NW;
    const int hp = (piece >> 2) * 64 + lane, oct = piece & 3;
    const int hy = hp / HWW, hx = hp - hy * HWW;
    const int iy = oy0 - dl + hy, ix = hx - dl;
    const bool ok = piece < npieces && hy < TY + 2 * dl && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
    hsrc[k] = ok ? ((b * a.IH + iy) * a.IW + ix) * a.hid + oct * 8 : -1;
  }
  const int nchunks = a.hid / 32;
  auto issue = [&](int c, int buf) {
    char* dst = smem + buf * BUF;
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
      const int piece = wid + k * NW;
      if (piece < npieces) {
        const void* src = hsrc[k] >= 0 ? (const void*)(a.h + hsrc[k] + c * 32) : (const void*)g_dwp_zero;
        __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(dst + (piece & 3) * PLANE + (piece >> 2) * 1024), 16, 0, 0);
      }
    }
    const char* wsrc = reinterpret_cast<const char*>(a.w) + (size_t)c * WB + lane * 16;
    for (int q = wid; q < NS + 1; q += NW)
      __builtin_amdgcn_global_load_lds(wsrc + q * 1024, (lds_ptr_t)(dst + HPP * 64 + q * 1024), 16, 0, 0);
  };

  const f16x8 h0 = {0, 0, 0, 0, 0, 0, 0, 0}, h6 = {6, 6, 6, 6, 6, 6, 6, 6};
  f32x4 acc[NS];
#pragma unroll
  for (int n = 0; n < NS; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int trow = dl * HWW * 16, tcol = dl * 16;  // tap strides (bytes, within an octet plane)

  // DMA instructions this wave issues per chunk (wave-uniform, fixed over chunks)
  int kw = 0;
#pragma unroll
  for (int k = 0; k < MAXP; ++k) kw += (wid + k * NW < npieces) ? 1 : 0;
  for (int q = wid; q < NS + 1; q += NW) ++kw;
#pragma unroll
  for (int s = 0; s < ST - 1; ++s)
    if (s < nchunks) issue(s, s);
  for (int c = 0; c < nchunks; ++c) {
    if (ST == 2 || c + ST - 2 >= nchunks) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {  // leave the newer chunks' DMAs (ST - 2 chunks x kw) in flight
      switch (kw * (ST - 2)) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      }
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + ST - 1 < nchunks) issue(c + ST - 1, (c + ST - 1) % ST);
    const char* Hb = smem + (c % ST) * BUF;
    const char* W = Hb + HPP * 64;
    const f16* wd = reinterpret_cast<const f16*>(W + NS * 1024);
    f16x8 d = *reinterpret_cast<const f16x8*>(wd + 9 * 32 + kq * 8);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const f16x8 v = *reinterpret_cast<const f16x8*>(Hb + dwbase + (t / 3) * trow + (t % 3) * tcol);
      d = v * *reinterpret_cast<const f16x8*>(wd + t * 32 + kq * 8) + d;
    }
    d = __builtin_elementwise_min(__builtin_elementwise_max(d, h0), h6);
    const char* Wl = W + lane * 16;
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const f16x8 af = *reinterpret_cast<const f16x8*>(Wl + n * 1024);
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, d, acc[n], 0, 0, 0);
    }
  }

  const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_bytes, 0x00020000);
#pragma unroll
  for (int pp = 0; pp < NS / 2; ++pp) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * pp][q]),
                                                      __float_as_uint(acc[2 * pp + 1][q]), false, false);
      v[q] = __uint_as_float(r[0]);
      v[q + 4] = __uint_as_float(r[1]);
    }
    const int n = (2 * pp + (kq & 1)) * 16 + (kq >> 1) * 8;
    const bool ok = pv && n < a.Cout;
    if (ok) {
      const float4 b0 = *reinterpret_cast<const float4*>(a.bp + n);
      const float4 b1 = *reinterpret_cast<const float4*>(a.bp + n + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
      if (a.res) {
        const bf16x8 rv = ld8(a.res + (size_t)m * a.Cout + n);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += (float)rv[q];
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (bf16)v[q];
    const int off = ok ? (m * a.Cout + n) * 2 : a.out_bytes;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), orsrc, off, 0, 0);
  }
}

template <int NS, int ST>
void launch_dwp_rows_st(const DPPArgs& a, int TY, int xcd, hipStream_t s) {
  const int HP = (TY + 2 * a.dil) * (a.OW + 2 * a.dil);
  const int HPP = (HP + 63) / 64 * 64;
  const int nw = (TY * a.OW + 15) / 16;
  const size_t lds = ST * ((size_t)HPP * 64 + (NS + 1) * 1024);
  if (nw > 16 || lds > 160 * 1024 || HPP / 16 > 4 * nw)
    throw std::invalid_argument("dw_proj_fused rows: tile too large");
  static bool attr = false;
  if (!attr) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&dw_proj_rows_kernel<NS, ST>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "dw_proj_rows attr");
    attr = true;
  }
  const int grid = a.B * cdiv(a.OH, TY);
  hipLaunchKernelGGL((dw_proj_rows_kernel<NS, ST>), dim3(grid), dim3(64 * nw), lds, s, a, TY, HPP, xcd);
  check_launch("dw_proj_rows");
}

template <int NS>
void launch_dwp_rows(const DPPArgs& a, int rows, hipStream_t s) {
  // rows = TY | stages << 8 | xcd << 12
  const int TY = rows & 0xff, st = (rows >> 8) & 0xf, xcd = (rows >> 12) & 1;
  if (st == 3) launch_dwp_rows_st<NS, 3>(a, TY, xcd, s);
  else if (st == 4) launch_dwp_rows_st<NS, 4>(a, TY, xcd, s);
  else launch_dwp_rows_st<NS, 2>(a, TY, xcd, s);
}

}  // namespace

void dw_proj_fused(const DwProjFusedParams& p, hipStream_t s) {
  if (p.hid % 32 || p.Cout % 16 || p.stride < 1) throw std::invalid_argument("dw_proj_fused: bad shape");
  const long long out_bytes = (long long)p.B * p.OH * p.OW * p.Cout * 2;
  if (out_bytes >= (1LL << 31) || (long long)p.B * p.IH * p.IW * p.hid >= (1LL << 31))
    throw std::invalid_argument("dw_proj_fused: tensor too large for 32-bit offsets");
  DPPArgs a{static_cast<const f16*>(p.h), static_cast<const f16*>(p.w), p.bp, p.res, p.out, p.B, p.IH, p.IW, p.hid, p.Cout, p.OH, p.OW, p.stride,
            p.dil, (int)out_bytes};
  if (p.rows > 0) {  // row-tile LDS-halo variant (stride 1)
    if (p.stride != 1) throw std::invalid_argument("dw_proj_fused rows: stride 1 only");
    switch (p.Cout / 16) {
      case 4: launch_dwp_rows<4>(a, p.rows, s); break;
      case 6: launch_dwp_rows<6>(a, p.rows, s); break;
      case 10: launch_dwp_rows<10>(a, p.rows, s); break;
      case 20: launch_dwp_rows<20>(a, p.rows, s); break;
      default: throw std::invalid_argument("dw_proj_fused: unsupported Cout");
    }
    return;
  }
  if (p.waves == 8) dispatch_dwp<8>(a, p.Cout / 16, s);
  else dispatch_dwp<4>(a, p.Cout / 16, s);
}

}  // namespace ssa
