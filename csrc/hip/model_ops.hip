// Memory-bound model kernels for gfx950: depthwise conv, fused preprocess+stem,
// max pool, global average pool, small matvec, fused bilinear upsample + argmax.
// All NHWC bf16 with 16-byte vector accesses along channels (8 bf16 per lane).
#include "common.h"
#include "kernels.h"

namespace ssa {

// ---------------------------------------------------------------- depthwise
// One lane = one output pixel x 8 channels; a wave covers 64 channel groups of
// consecutive pixels, so loads/stores are 16 B per lane and contiguous.
__global__ __launch_bounds__(256) void dw3x3_kernel(const bf16* __restrict__ in,
                                                    const float* __restrict__ w,
                                                    const float* __restrict__ bias,
                                                    bf16* __restrict__ out, int B, int IH, int IW,
                                                    int C, int OH, int OW, int stride, int dil,
                                                    int act) {
  const int CG = C >> 3;
  const long long total = (long long)B * OH * OW * CG;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % CG);
    long long pix = t / CG;
    const int ox = (int)(pix % OW);
    pix /= OW;
    const int oy = (int)(pix % OH);
    const int b = (int)(pix / OH);
    const int c = cg * 8;
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = bias[c + q];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * stride + (ky - 1) * dil;
      if (iy < 0 || iy >= IH) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox * stride + (kx - 1) * dil;
        if (ix < 0 || ix >= IW) continue;
        const bf16x8 v = ld8(in + (((long long)b * IH + iy) * IW + ix) * C + c);
        const float4 w0 = *reinterpret_cast<const float4*>(w + (ky * 3 + kx) * C + c);
        const float4 w1 = *reinterpret_cast<const float4*>(w + (ky * 3 + kx) * C + c + 4);
        acc[0] += (float)v[0] * w0.x; acc[1] += (float)v[1] * w0.y;
        acc[2] += (float)v[2] * w0.z; acc[3] += (float)v[3] * w0.w;
        acc[4] += (float)v[4] * w1.x; acc[5] += (float)v[5] * w1.y;
        acc[6] += (float)v[6] * w1.z; acc[7] += (float)v[7] * w1.w;
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (bf16)apply_act(acc[q], act);
    st8(out + t * 8, o);
  }
}

// Strip variant: one lane = PX consecutive output pixels of one row x 8 channels,
// stride / dilation compile-time, so the (PX-1)*S + 2D + 1 input columns of a
// kernel row are loaded once and shared by the strip's taps (6 loads instead of
// 12 per row at S1 D1, 9 instead of 12 at S2), weights are loaded once per strip,
// and all index math is 32-bit (the flat 64-bit div/mod chain above costs more
// than the arithmetic on the 33x33 maps).
template <int S, int D, int PX>
__global__ __launch_bounds__(256) void dw3x3_strip_kernel(const bf16* __restrict__ in,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          bf16* __restrict__ out, int B, int IH,
                                                          int IW, int C, int OH, int OW, int act) {
  constexpr int NC = (PX - 1) * S + 2 * D + 1;
  const int CG = C >> 3;
  const int SX = (OW + PX - 1) / PX;
  const int total = B * OH * SX * CG;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int cg = t % CG;
  int r = t / CG;
  const int sx = r % SX;
  r /= SX;
  const int oy = r % OH, b = r / OH;
  const int c = cg * 8, ox0 = sx * PX;
  float acc[PX][8];
  {
    const float4 b0 = *reinterpret_cast<const float4*>(bias + c);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + c + 4);
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      acc[p][0] = b0.x; acc[p][1] = b0.y; acc[p][2] = b0.z; acc[p][3] = b0.w;
      acc[p][4] = b1.x; acc[p][5] = b1.y; acc[p][6] = b1.z; acc[p][7] = b1.w;
    }
  }
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * S + (ky - 1) * D;
    if (iy < 0 || iy >= IH) continue;
    const bf16* row = in + ((size_t)(b * IH + iy) * IW) * C + c;
    bf16x8 col[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int ix = ox0 * S - D + j;
      col[j] = (ix >= 0 && ix < IW) ? ld8(row + (size_t)ix * C) : zero8();
    }
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const float4 w0 = *reinterpret_cast<const float4*>(w + (ky * 3 + kx) * C + c);
      const float4 w1 = *reinterpret_cast<const float4*>(w + (ky * 3 + kx) * C + c + 4);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        const bf16x8 v = col[p * S + kx * D];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[p][q] += (float)v[q] * wv[q];
      }
    }
  }
  bf16* op = out + ((size_t)(b * OH + oy) * OW + ox0) * C + c;
#pragma unroll
  for (int p = 0; p < PX; ++p) {
    if (ox0 + p >= OW) break;
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (bf16)apply_act(acc[p][q], act);
    st8(op + (size_t)p * C, o);
  }
}

void depthwise3x3(const bf16* in, const float* w, const float* bias, bf16* out, int B, int IH,
                  int IW, int C, int OH, int OW, int stride, int dil, int act, hipStream_t s) {
  if (C % 8) throw std::invalid_argument("depthwise3x3: C must be a multiple of 8");
  constexpr int PX = 4;
  const long long strip_total = (long long)B * OH * ((OW + PX - 1) / PX) * (C / 8);
  if (strip_total < (1LL << 31) && (long long)B * IH * IW * C < (1LL << 40)) {
    const int grid = cdiv(strip_total, 256);
#define DWS(S_, D_)                                                                              \
    if (stride == S_ && dil == D_) {                                                             \
      hipLaunchKernelGGL((dw3x3_strip_kernel<S_, D_, PX>), dim3(grid), dim3(256), 0, s, in, w,   \
                         bias, out, B, IH, IW, C, OH, OW, act);                                  \
      check_launch("depthwise3x3 strip");                                                        \
      return;                                                                                    \
    }
    DWS(1, 1) DWS(1, 2) DWS(2, 1) DWS(1, 4)
#undef DWS
  }
  const long long total = (long long)B * OH * OW * (C / 8);
  const int grid = (int)std::min<long long>(cdiv(total, 256), 256LL * 32);
  hipLaunchKernelGGL(dw3x3_kernel, dim3(grid), dim3(256), 0, s, in, w, bias, out, B, IH, IW, C,
                     OH, OW, stride, dil, act);
  check_launch("depthwise3x3");
}

// ---------------------------------------------------------------- stem
// One lane = one output pixel x all Cout channels. The letterbox LUT turns the
// uint8 camera frame into the normalised model input on the fly, so the
// preprocessed 513x513x3 tensor is never materialised. Weights live in LDS.
template <int COUT>
__global__ __launch_bounds__(256) void stem_kernel(const uint8_t* __restrict__ frames,
                                                   const int32_t* __restrict__ lut_x,
                                                   const int32_t* __restrict__ lut_y,
                                                   const float* __restrict__ w,
                                                   const float* __restrict__ bias,
                                                   void* __restrict__ outv, int B, int Hc, int Wc,
                                                   int H, int W, int OH, int OW, int K,
                                                   int stride, int act, float out_inv_scale) {
  extern __shared__ __attribute__((aligned(16))) float sw[];  // [K*K*3][COUT] + bias
  const int nw = K * K * 3 * COUT;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) sw[i] = w[i];
  for (int i = threadIdx.x; i < COUT; i += blockDim.x) sw[nw + i] = bias[i];
  __syncthreads();
  const long long total = (long long)B * OH * OW;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int ox = (int)(t % OW);
  const int oy = (int)((t / OW) % OH);
  const int b = (int)(t / ((long long)OW * OH));
  float acc[COUT];
#pragma unroll
  for (int n = 0; n < COUT; ++n) acc[n] = sw[nw + n];
  const int pad = K / 2;
  const uint8_t* fb = frames + (long long)b * Hc * Wc * 3;
  for (int ky = 0; ky < K; ++ky) {
    const int y = oy * stride + ky - pad;
    if (y < 0 || y >= H) continue;  // conv zero padding (outside the model input)
    const int sy = lut_y[y];
    for (int kx = 0; kx < K; ++kx) {
      const int x = ox * stride + kx - pad;
      if (x < 0 || x >= W) continue;
      const int sx = lut_x[x];
      float rgb[3];
      if (sy >= 0 && sx >= 0) {
        const uint8_t* px = fb + ((long long)sy * Wc + sx) * 3;
        rgb[0] = px[2] * (1.f / 127.5f) - 1.f;  // BGR -> RGB
        rgb[1] = px[1] * (1.f / 127.5f) - 1.f;
        rgb[2] = px[0] * (1.f / 127.5f) - 1.f;
      } else {  // letterbox padding: uint8 zero -> -1
        rgb[0] = rgb[1] = rgb[2] = -1.f;
      }
      const float* wt = sw + ((ky * K + kx) * 3) * COUT;
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int n = 0; n < COUT; ++n) acc[n] += rgb[c] * wt[c * COUT + n];
    }
  }
  if (out_inv_scale > 0.f) {  // int8 output for the int8 pipelines
    int8_t* op = static_cast<int8_t*>(outv) + t * COUT;
#pragma unroll
    for (int n = 0; n < COUT; n += 8) {
      signed char q8[8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        q8[q] = (signed char)fminf(fmaxf(rintf(apply_act(acc[n + q], act) * out_inv_scale), -127.f), 127.f);
      *reinterpret_cast<int2*>(op + n) = *reinterpret_cast<int2*>(q8);
    }
    return;
  }
  bf16* op = static_cast<bf16*>(outv) + t * COUT;
#pragma unroll
  for (int n = 0; n < COUT; n += 8) {
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (bf16)apply_act(acc[n + q], act);
    st8(op + n, o);
  }
}

void stem_conv(const uint8_t* frames, const int32_t* lut_x, const int32_t* lut_y, const float* w,
               const float* bias, void* out, int B, int Hc, int Wc, int H, int W, int OH, int OW,
               int Cout, int K, int stride, int act, hipStream_t s, float out_inv_scale) {
  const long long total = (long long)B * OH * OW;
  const size_t lds = (size_t)(K * K * 3 * Cout + Cout) * sizeof(float);
  const int grid = cdiv(total, 256);
#define STEM_CASE(C)                                                                          \
  case C:                                                                                     \
    hipLaunchKernelGGL(stem_kernel<C>, dim3(grid), dim3(256), lds, s, frames, lut_x, lut_y, w, \
                       bias, out, B, Hc, Wc, H, W, OH, OW, K, stride, act, out_inv_scale);   \
    break;
  switch (Cout) {
    STEM_CASE(16)
    STEM_CASE(24)
    STEM_CASE(32)
    STEM_CASE(48)
    STEM_CASE(64)
    default:
      throw std::invalid_argument("stem_conv: unsupported Cout");
  }
#undef STEM_CASE
  check_launch("stem_conv");
}

// ---------------------------------------------------------------- MFMA stem
// The same conv on v_mfma_f32_16x16x16_bf16 (the dense stem of DeepLabv3-ResNet50:
// 7x7 s2, 3 -> 64 at 513^2 per frame): a workgroup owns a TY x TX output tile,
// gathers the letterboxed input region under it ONCE into LDS as bf16 RGB0 pixels
// (8 bytes: the stem_block0 layout), and every 16 output pixels x 16 channels are
// KG MFMAs over K = taps x 4 channels (lane kq of MFMA m holds tap 4m + kq: one
// 8-byte LDS read). The per-lane kernel above re-gathers 49 camera pixels (LUTs +
// 3 byte loads each) for every output pixel and runs 9.4k fp32 FMAs per pixel.
typedef short s16x4m __attribute__((ext_vector_type(4)));

struct SMArgs {
  const uint8_t* frames; const int32_t* lut_x; const int32_t* lut_y;
  const bf16* w;      // [Cout][KG * 16], K = tap * 4 + c (c = 3 and taps >= K*K zero)
  const float* bias;  // [Cout]
  void* out;
  int B, Hc, Wc, H, W, OH, OW, K, stride, act, TY, TX, tiles_y, tiles_x;
  float out_inv_scale;  // > 0: int8 output
};

template <int NSUB, int KG, int GPW>
__global__ __launch_bounds__(256) void stem_mfma_kernel(SMArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* IN = reinterpret_cast<bf16*>(smem);
  const int IHT = (a.TY - 1) * a.stride + a.K, IWT = (a.TX - 1) * a.stride + a.K;
  const int ntile = a.tiles_y * a.tiles_x;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bid / ntile, t = bid % ntile;
  const int oy0 = (t / a.tiles_x) * a.TY, ox0 = (t % a.tiles_x) * a.TX;
  const int iy0 = oy0 * a.stride - a.K / 2, ix0 = ox0 * a.stride - a.K / 2;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const float inv_tx = 1.f / a.TX;
  const uint8_t* fb = a.frames + (size_t)b * a.Hc * a.Wc * 3;
  gather_letterbox_rgb0<6, 256>(IN, fb, a.lut_x, a.lut_y, a.Wc, a.H, a.W, iy0, ix0, IHT, IWT, tid);
  s16x4m wf[NSUB][KG];
  f32x4 bs[NSUB];
#pragma unroll
  for (int sub = 0; sub < NSUB; ++sub) {
#pragma unroll
    for (int m = 0; m < KG; ++m)
      wf[sub][m] = *reinterpret_cast<const s16x4m*>(a.w + (size_t)(sub * 16 + r16) * (KG * 16) + m * 16 + kq * 4);
    bs[sub] = *reinterpret_cast<const f32x4*>(a.bias + sub * 16 + kq * 4);
  }
  int toff[KG];
#pragma unroll
  for (int m = 0; m < KG; ++m) {
    const int tp = m * 4 + kq;
    toff[m] = tp < a.K * a.K ? ((tp / a.K) * IWT + tp % a.K) * 4 : -1;
  }
  __syncthreads();
  const s16x4m zs = {0, 0, 0, 0};
  const int Cout = NSUB * 16;
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    const int p = (wid * GPW + g) * 16 + r16;
    const int py = (int)(((float)p + 0.5f) * inv_tx), px = p - py * a.TX;
    const int oy = oy0 + py, ox = ox0 + px;
    const bool valid = p < a.TY * a.TX && oy < a.OH && ox < a.OW;
    const int base = valid ? (py * a.stride * IWT + px * a.stride) * 4 : 0;
    s16x4m xf[KG];
#pragma unroll
    for (int m = 0; m < KG; ++m)
      xf[m] = toff[m] >= 0 ? *reinterpret_cast<const s16x4m*>(IN + base + toff[m]) : zs;
    const size_t pix = ((size_t)b * a.OH + oy) * a.OW + ox;
#pragma unroll
    for (int sub = 0; sub < NSUB; ++sub) {
      f32x4 acc = bs[sub];
#pragma unroll
      for (int m = 0; m < KG; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wf[sub][m], xf[m], acc, 0, 0, 0);
      if (!valid) continue;
      const int n = sub * 16 + kq * 4;
      if (a.out_inv_scale > 0.f) {
        char4 o;
        o.x = (signed char)fminf(fmaxf(rintf(apply_act(acc[0], a.act) * a.out_inv_scale), -127.f), 127.f);
        o.y = (signed char)fminf(fmaxf(rintf(apply_act(acc[1], a.act) * a.out_inv_scale), -127.f), 127.f);
        o.z = (signed char)fminf(fmaxf(rintf(apply_act(acc[2], a.act) * a.out_inv_scale), -127.f), 127.f);
        o.w = (signed char)fminf(fmaxf(rintf(apply_act(acc[3], a.act) * a.out_inv_scale), -127.f), 127.f);
        *reinterpret_cast<char4*>(static_cast<int8_t*>(a.out) + pix * Cout + n) = o;
      } else {
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)apply_act(acc[q], a.act);
        *reinterpret_cast<bf16x4*>(static_cast<bf16*>(a.out) + pix * Cout + n) = o;
      }
    }
  }
}

// Wave-per-channel-block variant (round 4, the 7x7 stem of config 4): wave w computes
// output channels 16w .. 16w + 15 for EVERY pixel group of the tile, so it holds one
// channel block's 13 weight fragments (26 VGPRs) instead of all four (104): the
// all-blocks kernel above needs 180 VGPRs, i.e. 2 workgroups per CU, and spends its
// time waiting on the gather with nothing else resident (328 us per 8 frames at 1025^2,
// 2.4 % of the MFMA peak, profiles/r4_config4_roofline.txt). The price is 4x the LDS
// reads of the input fragments (each wave reads every group's), which LDS absorbs; the
// smaller per-wave state also lets a workgroup own bigger tiles (up to 32 x 32 pixels),
// which cuts the gathered halo per output pixel.
template <int KG>
__global__ __launch_bounds__(256) void stem_mfma_ws_kernel(SMArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* IN = reinterpret_cast<bf16*>(smem);
  const int IHT = (a.TY - 1) * a.stride + a.K, IWT = (a.TX - 1) * a.stride + a.K;
  const int ntile = a.tiles_y * a.tiles_x;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bid / ntile, t = bid % ntile;
  const int oy0 = (t / a.tiles_x) * a.TY, ox0 = (t % a.tiles_x) * a.TX;
  const int iy0 = oy0 * a.stride - a.K / 2, ix0 = ox0 * a.stride - a.K / 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int sub = __builtin_amdgcn_readfirstlane(tid >> 6);  // this wave's 16 channels
  const int r16 = lane & 15, kq = lane >> 4;
  const float inv_tx = 1.f / a.TX;
  const uint8_t* fb = a.frames + (size_t)b * a.Hc * a.Wc * 3;
  gather_letterbox_rgb0<6, 256>(IN, fb, a.lut_x, a.lut_y, a.Wc, a.H, a.W, iy0, ix0, IHT, IWT, tid);
  s16x4m wf[KG];
#pragma unroll
  for (int m = 0; m < KG; ++m)
    wf[m] = *reinterpret_cast<const s16x4m*>(a.w + (size_t)(sub * 16 + r16) * (KG * 16) + m * 16 + kq * 4);
  const f32x4 bs = *reinterpret_cast<const f32x4*>(a.bias + sub * 16 + kq * 4);
  // taps past K*K (the last fragment's padding) read tap 0's pixel: their weights are
  // zero, and an unconditional read lets all KG LDS reads issue before the MFMA chain (an
  // exec-masked read per fragment serialised read -> wait -> MFMA 13 times per group)
  int toff[KG];
#pragma unroll
  for (int m = 0; m < KG; ++m) {
    const int tp = m * 4 + kq;
    toff[m] = tp < a.K * a.K ? ((tp / a.K) * IWT + tp % a.K) * 4 : 0;
  }
  __syncthreads();
  const int Cout = 64;
  const int n = sub * 16 + kq * 4;
  const int groups = (a.TY * a.TX + 15) / 16;
#pragma unroll 2
  for (int g = 0; g < groups; ++g) {
    const int p = g * 16 + r16;
    const int py = (int)(((float)p + 0.5f) * inv_tx), px = p - py * a.TX;
    const int oy = oy0 + py, ox = ox0 + px;
    const bool valid = p < a.TY * a.TX && oy < a.OH && ox < a.OW;
    const int base = valid ? (py * a.stride * IWT + px * a.stride) * 4 : 0;
    s16x4m xf[KG];
#pragma unroll
    for (int m = 0; m < KG; ++m) xf[m] = *reinterpret_cast<const s16x4m*>(IN + base + toff[m]);
    f32x4 acc = bs;
#pragma unroll
    for (int m = 0; m < KG; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wf[m], xf[m], acc, 0, 0, 0);
    if (!valid) continue;
    const size_t pix = ((size_t)b * a.OH + oy) * a.OW + ox;
    if (a.out_inv_scale > 0.f && a.act == ACT_RELU) {
      // relu + int8: the codes are rint(clamp(acc * s, 0, 127)) -- one med3 and one rounding
      // pack per value (v_cvt_pk_u8_f32, nearest even like rintf; clamping to integer bounds
      // before or after the rounding gives the same code), non-negative so the unsigned
      // bytes are the signed ones. The float chain below took ~7 VALU per value.
      unsigned w = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(acc[q] * a.out_inv_scale, 0.f, 127.f), q, w);
      *reinterpret_cast<unsigned*>(static_cast<int8_t*>(a.out) + pix * Cout + n) = w;
    } else if (a.out_inv_scale > 0.f) {
      char4 o;
      o.x = (signed char)fminf(fmaxf(rintf(apply_act(acc[0], a.act) * a.out_inv_scale), -127.f), 127.f);
      o.y = (signed char)fminf(fmaxf(rintf(apply_act(acc[1], a.act) * a.out_inv_scale), -127.f), 127.f);
      o.z = (signed char)fminf(fmaxf(rintf(apply_act(acc[2], a.act) * a.out_inv_scale), -127.f), 127.f);
      o.w = (signed char)fminf(fmaxf(rintf(apply_act(acc[3], a.act) * a.out_inv_scale), -127.f), 127.f);
      *reinterpret_cast<char4*>(static_cast<int8_t*>(a.out) + pix * Cout + n) = o;
    } else {
      bf16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = (bf16)apply_act(acc[q], a.act);
      *reinterpret_cast<bf16x4*>(static_cast<bf16*>(a.out) + pix * Cout + n) = o;
    }
  }
}

void stem_mfma(const uint8_t* frames, const int32_t* lut_x, const int32_t* lut_y, const bf16* w,
               const float* bias, void* out, int B, int Hc, int Wc, int H, int W, int OH, int OW,
               int Cout, int K, int stride, int act, float out_inv_scale, int TY, int TX,
               hipStream_t s, int mode) {
  if (mode == 1) {  // wave per 16-channel block: 7x7 / 64-channel stem only
    if (Cout != 64 || (K * K + 3) / 4 != 13) throw std::invalid_argument("stem_mfma ws: (Cout, K) must be (64, 7)");
    if (TY < 1 || TX < 1 || TY * TX > 1024) throw std::invalid_argument("stem_mfma ws: bad tile");
    const size_t lds = (size_t)((TY - 1) * stride + K) * ((TX - 1) * stride + K) * 8;
    if (lds > 64 * 1024) throw std::invalid_argument("stem_mfma ws: tile too large");
    SMArgs a{frames, lut_x, lut_y, w, bias, out, B, Hc, Wc, H, W, OH, OW, K, stride, act, TY, TX,
             cdiv(OH, TY), cdiv(OW, TX), out_inv_scale};
    hipLaunchKernelGGL((stem_mfma_ws_kernel<13>), dim3(B * a.tiles_y * a.tiles_x), dim3(256), lds, s, a);
    check_launch("stem_mfma ws");
    return;
  }
  if (mode != 0) throw std::invalid_argument("stem_mfma: mode must be 0 or 1");
  if (TY < 1 || TX < 1 || TY * TX > 256 || TX > 120) throw std::invalid_argument("stem_mfma: bad tile");
  const int IHT = (TY - 1) * stride + K, IWT = (TX - 1) * stride + K;
  const size_t lds = (size_t)IHT * IWT * 8;
  if (lds > 64 * 1024) throw std::invalid_argument("stem_mfma: tile too large");
  SMArgs a{frames, lut_x, lut_y, w, bias, out, B, Hc, Wc, H, W, OH, OW, K, stride, act, TY, TX,
           cdiv(OH, TY), cdiv(OW, TX), out_inv_scale};
  const int grid = B * a.tiles_y * a.tiles_x;
  const int groups = (TY * TX + 15) / 16;
  const int kg = (K * K + 3) / 4;
#define SM(NS, KGV, G) hipLaunchKernelGGL((stem_mfma_kernel<NS, KGV, G>), dim3(grid), dim3(256), lds, s, a)
  if (Cout == 64 && kg == 13) {
    if (groups <= 4) SM(4, 13, 1); else if (groups <= 8) SM(4, 13, 2); else SM(4, 13, 4);
  } else if (Cout == 32 && kg == 3) {
    if (groups <= 4) SM(2, 3, 1); else if (groups <= 8) SM(2, 3, 2); else SM(2, 3, 4);
  } else {
    throw std::invalid_argument("stem_mfma: (Cout, K) must be (64, 7) or (32, 3)");
  }
#undef SM
  check_launch("stem_mfma");
}

// ---------------------------------------------------------------- max pool
__global__ void maxpool_kernel(const bf16* __restrict__ in, bf16* __restrict__ out, int B, int IH,
                               int IW, int C, int OH, int OW) {
  const int CG = C >> 3;
  const long long total = (long long)B * OH * OW * CG;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int cg = (int)(t % CG);
  long long pix = t / CG;
  const int ox = (int)(pix % OW);
  pix /= OW;
  const int oy = (int)(pix % OH);
  const int b = (int)(pix / OH);
  float m[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) m[q] = -3.0e38f;
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * 2 + ky - 1;
    if (iy < 0 || iy >= IH) continue;
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ox * 2 + kx - 1;
      if (ix < 0 || ix >= IW) continue;
      const bf16x8 v = ld8(in + (((long long)b * IH + iy) * IW + ix) * C + cg * 8);
#pragma unroll
      for (int q = 0; q < 8; ++q) m[q] = fmaxf(m[q], (float)v[q]);
    }
  }
  bf16x8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = (bf16)m[q];
  st8(out + t * 8, o);
}

void maxpool3x3s2(const bf16* in, bf16* out, int B, int IH, int IW, int C, int OH, int OW,
                  hipStream_t s) {
  const long long total = (long long)B * OH * OW * (C / 8);
  hipLaunchKernelGGL(maxpool_kernel, dim3(cdiv(total, 256)), dim3(256), 0, s, in, out, B, IH, IW,
                     C, OH, OW);
  check_launch("maxpool3x3s2");
}

// ---------------------------------------------------------------- GAP
// Two passes so the reduction fills the chip: grid (B, S slices of the pixels,
// channel blocks); each lane owns 8 channels, the 4 waves of a block split the
// slice's pixels and reduce through LDS into part[b][slice][C]; a tiny second
// kernel sums the slices (deterministic, no float atomics).
// 32 slices and four 16-byte loads in flight per lane: with 16 slices and one load per
// iteration each wave walked 17 pixels through 17 dependent L2/HBM round trips (10 us at
// B = 32, 8 us at B = 1 where the grid is only 16 workgroups: r8l / r8p step traces).
constexpr int kGapSlices = 32;

__global__ __launch_bounds__(256) void gap_partial_kernel(const bf16* __restrict__ in,
                                                          float* __restrict__ part, int HW, int C) {
  const int b = blockIdx.x, sl = blockIdx.y;
  const int CG = C >> 3;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int cg = blockIdx.z * 64 + lane;
  __shared__ float red[4][64][8];
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int p0 = (int)((long long)HW * sl / kGapSlices), p1 = (int)((long long)HW * (sl + 1) / kGapSlices);
  if (cg < CG) {
    const bf16* base = in + (long long)b * HW * C + cg * 8;
    int p = p0 + wid;
    for (; p + 12 < p1; p += 16) {  // this wave's next 4 pixels: all loads issued first
      bf16x8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ld8(base + (long long)(p + 4 * u) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += (float)v[u][q];
    }
    for (; p < p1; p += 4) {
      const bf16x8 v = ld8(base + (long long)p * C);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += (float)v[q];
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) red[wid][lane][q] = acc[q];
  __syncthreads();
  if (wid == 0 && cg < CG) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      part[((long long)b * kGapSlices + sl) * C + cg * 8 + q] =
          red[0][lane][q] + red[1][lane][q] + red[2][lane][q] + red[3][lane][q];
  }
}

__global__ void gap_reduce_kernel(const float* __restrict__ part, float* __restrict__ out, int B,
                                  int HW, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i % C;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kGapSlices; ++k) s += part[((long long)b * kGapSlices + k) * C + c];
  out[i] = s / (float)HW;
}

size_t gap_workspace_floats(int B, int C) { return (size_t)B * kGapSlices * C; }

// ---------------------------------------------------------------- device -> pinned host
// The per-step packed records (B x 1.3 KB) are written straight into pinned host memory
// (hipHostMalloc: device-addressable, coherent) by a kernel on the stream that produced
// them. hipMemcpyAsync D2H here stalled the host thread for up to ~6 ms in the lag-2
// pipeline (scripts/lag_timeline.py: one copy_ call per ~20 steps blocked until the
// result stream drained); a kernel launch never blocks the host.
__global__ __launch_bounds__(256) void copy_to_host_kernel(const uint4* __restrict__ src,
                                                           uint4* __restrict__ dst, long long n16,
                                                           const uint32_t* __restrict__ src4,
                                                           uint32_t* __restrict__ dst4, long long n4) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long k = i; k < n16; k += stride) dst[k] = src[k];
  for (long long k = i; k < n4; k += stride) dst4[k] = src4[k];
}

void copy_to_host(const void* src, void* dst, long long nbytes, hipStream_t s) {
  if (nbytes % 4) throw std::invalid_argument("copy_to_host: nbytes % 4 == 0 required");
  const bool al = ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0);
  const long long n16 = al ? nbytes / 16 : 0;
  const long long tail = nbytes - n16 * 16;
  const auto* s4 = reinterpret_cast<const uint32_t*>(static_cast<const char*>(src) + n16 * 16);
  auto* d4 = reinterpret_cast<uint32_t*>(static_cast<char*>(dst) + n16 * 16);
  const long long work = n16 > tail / 4 ? n16 : tail / 4;
  const int grid = (int)std::min<long long>(64, std::max<long long>(1, cdiv(work, 256)));
  hipLaunchKernelGGL(copy_to_host_kernel, dim3(grid), dim3(256), 0, s, static_cast<const uint4*>(src),
                     static_cast<uint4*>(dst), n16, s4, d4, tail / 4);
  check_launch("copy_to_host");
}

// dst row r = [a row r | b row r] (4-byte words). a/b may be device or pinned host memory:
// the records + frame metadata of one step become ONE send buffer, so the RCCL gather to
// rank 0 is a single collective and the metadata needs no H2D hipMemcpyAsync of its own.
__global__ __launch_bounds__(256) void pack_rows_kernel(uint32_t* __restrict__ dst,
                                                        const uint32_t* __restrict__ a, int aw,
                                                        const uint32_t* __restrict__ b, int bw,
                                                        int rows) {
  const int w = aw + bw;
  const long long n = (long long)rows * w;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / w;
    const int c = (int)(i - r * w);
    dst[i] = c < aw ? a[r * aw + c] : b[r * bw + (c - aw)];
  }
}

void pack_rows(void* dst, const void* a, int a_words, const void* b, int b_words, int rows,
               hipStream_t s) {
  if (rows <= 0 || a_words < 0 || b_words < 0) throw std::invalid_argument("pack_rows: bad shape");
  const long long n = (long long)rows * (a_words + b_words);
  const int grid = (int)std::min<long long>(64, std::max<long long>(1, cdiv(n, 256)));
  hipLaunchKernelGGL(pack_rows_kernel, dim3(grid), dim3(256), 0, s, static_cast<uint32_t*>(dst),
                     static_cast<const uint32_t*>(a), a_words, static_cast<const uint32_t*>(b),
                     b_words, rows);
  check_launch("pack_rows");
}

void global_avgpool(const bf16* in, float* out, float* ws, int B, int HW, int C, hipStream_t s) {
  hipLaunchKernelGGL(gap_partial_kernel, dim3(B, kGapSlices, cdiv(C / 8, 64)), dim3(256), 0, s, in,
                     ws, HW, C);
  hipLaunchKernelGGL(gap_reduce_kernel, dim3(cdiv((long long)B * C, 256)), dim3(256), 0, s, ws, out,
                     B, HW, C);
  check_launch("global_avgpool");
}

// ---------------------------------------------------------------- matvec
// One wave per (b, n): lanes split K, shuffle-reduce across the 64-lane wave.
__global__ __launch_bounds__(256) void matvec_kernel(const float* __restrict__ x,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ bias,
                                                     float* __restrict__ out, int B, int N, int K,
                                                     int act) {
  const int lane = threadIdx.x & 63;
  const long long item = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= (long long)B * N) return;
  const int b = (int)(item / N), n = (int)(item % N);
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += w[(long long)n * K + k] * x[(long long)b * K + k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[item] = apply_act(s + (bias ? bias[n] : 0.f), act);
}

// Epilogue of a library GEMM (the ASPP projection on hipBLASLt):
//   out[m, n] = act(in[m, n] + bias[n] + img_bias[m / HW][n]), bf16, 8 channels per thread
__global__ __launch_bounds__(256) void bias_act_kernel(const bf16* __restrict__ in,
                                                       const float* __restrict__ bias,
                                                       const float* __restrict__ img_bias,
                                                       bf16* __restrict__ out, int M, int N,
                                                       int HW, int act) {
  // 32-bit index math (host checks M * N < 2^31): the 64-bit divisions of a naive
  // version cost more than the memory traffic
  const int NG = N >> 3;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * NG) return;
  const int m = t / NG;
  const int n = (t - m * NG) * 8;
  const bf16x8 v = ld8(in + (size_t)m * N + n);
  float4 b0 = *reinterpret_cast<const float4*>(bias + n), b1 = *reinterpret_cast<const float4*>(bias + n + 4);
  if (img_bias) {
    const float* ib = img_bias + (size_t)(m / HW) * N + n;
    const float4 i0 = *reinterpret_cast<const float4*>(ib), i1 = *reinterpret_cast<const float4*>(ib + 4);
    b0.x += i0.x; b0.y += i0.y; b0.z += i0.z; b0.w += i0.w;
    b1.x += i1.x; b1.y += i1.y; b1.z += i1.z; b1.w += i1.w;
  }
  const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  bf16x8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = (bf16)apply_act((float)v[q] + bb[q], act);
  st8(out + (size_t)m * N + n, o);
}

void bias_act(const bf16* in, const float* bias, const float* img_bias, bf16* out, long long M, int N,
              int HW, int act, hipStream_t s) {
  if (N % 8 || HW < 1) throw std::invalid_argument("bias_act: N % 8 == 0 and HW >= 1 required");
  if (M * (long long)N >= (1LL << 31)) throw std::invalid_argument("bias_act: matrix too large");
  hipLaunchKernelGGL(bias_act_kernel, dim3(cdiv(M * (N / 8), 256)), dim3(256), 0, s, in, bias, img_bias,
                     out, (int)M, N, HW, act);
  check_launch("bias_act");
}

void matvec(const float* x, const float* w, const float* bias, float* out, int B, int N, int K,
            int act, hipStream_t s) {
  // (a batched one-wave-per-n form that read each weight row once measured slower here:
  // 23.0 vs 18.0 us for B = 8, N = 256, K = 2048 -- 256 waves leave the chip latency-bound)
  hipLaunchKernelGGL(matvec_kernel, dim3(cdiv((long long)B * N, 4)), dim3(256), 0, s, x, w, bias,
                     out, B, N, K, act);
  check_launch("matvec");
}

// ---------------------------------------------------------------- ASPP image-pooling branch
// The whole branch after the pixel sums in ONE workgroup per image (was gap_reduce +
// two matvec launches, ~3 x 10 us of launch-bound kernels per step for ~0.3 MFLOP):
//   gap[k]      = sum_s part[b][s][k] / HW                    (LDS)
//   pooled[n]   = relu(sum_k w1t[k][n] gap[k] + b1[n])         (LDS)
//   img_bias[n] = sum_k w2t[k][n] pooled[k]                   (-> projection epilogue)
// Weights are host-transposed [K][N]. Each of the 1024 threads owns 4 consecutive
// outputs (one float4 weight load per k) and a K slice; the slices are summed through
// LDS. A first version gave each thread whole K=320 dot products: ~80 dependent L2
// round trips per thread, 30 us for one image (profiles/r2_b1 trace).
constexpr int kPoolMaxC = 2048, kPoolMaxN = 512;

__device__ __forceinline__ float4 pool_slice(const float* __restrict__ wt, const float* s_x, int k0,
                                             int k1, int N, int q) {
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
  int k = k0;
  for (; k + 2 <= k1; k += 2) {
    const float4 w0 = *reinterpret_cast<const float4*>(wt + (size_t)k * N + 4 * q);
    const float4 w1 = *reinterpret_cast<const float4*>(wt + (size_t)(k + 1) * N + 4 * q);
    const float x0 = s_x[k], x1 = s_x[k + 1];
    a0.x += w0.x * x0; a0.y += w0.y * x0; a0.z += w0.z * x0; a0.w += w0.w * x0;
    a1.x += w1.x * x1; a1.y += w1.y * x1; a1.z += w1.z * x1; a1.w += w1.w * x1;
  }
  if (k < k1) {
    const float4 w0 = *reinterpret_cast<const float4*>(wt + (size_t)k * N + 4 * q);
    const float x0 = s_x[k];
    a0.x += w0.x * x0; a0.y += w0.y * x0; a0.z += w0.z * x0; a0.w += w0.w * x0;
  }
  return make_float4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w);
}

template <int kPoolThreads>
__global__ __launch_bounds__(kPoolThreads) void aspp_pool_kernel(const float* __restrict__ part,
                                                                 const float* __restrict__ w1t,
                                                                 const float* __restrict__ b1,
                                                                 const float* __restrict__ w2t,
                                                                 float* __restrict__ img_bias, int HW,
                                                                 int C, int N, float* dbg, int mode) {
  __shared__ float s_gap[kPoolMaxC];
  if (mode & 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __shared__ float s_pool[kPoolMaxN];
  __shared__ float4 s_red[kPoolThreads];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float inv = 1.f / (float)HW;
  const float* pb = part + (size_t)b * kGapSlices * C;
  for (int k = tid; k < C; k += kPoolThreads) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < kGapSlices; ++q) s += pb[(size_t)q * C + k];
    s_gap[k] = s * inv;
  }
  const int nq = N >> 2;                    // float4 output columns
  const int nks = kPoolThreads / nq;        // K slices
  const int q = tid % nq, ks = tid / nq;
  __syncthreads();
  // debug (scripts/debug_pool.py): per image [C gap | N pool | 4 x 1024 float4 stage views]
  const size_t dstride = (size_t)C + N + 4 * 4 * kPoolThreads;
  float* dimg = dbg ? dbg + (size_t)b * dstride : nullptr;
  float4* dv = dbg ? reinterpret_cast<float4*>(dimg + C + N) : nullptr;
  if (dbg)
    for (int k = tid; k < C; k += kPoolThreads) dimg[k] = s_gap[k];
  {
    const int per = (C + nks - 1) / nks;
    const int k0 = min(C, ks * per), k1 = min(C, k0 + per);
    if (ks < nks) {
      const float4 r = pool_slice(w1t, s_gap, k0, k1, N, q);
      s_red[ks * nq + q] = r;
      if (dbg) dv[tid] = r;
    }
  }
  __syncthreads();
  if (tid < nq) {
    float4 s = s_red[tid];
    if (dbg) dv[kPoolThreads + tid] = s;
    for (int j = 1; j < nks; ++j) {
      const float4 v = s_red[j * nq + tid];
      if (dbg) dv[kPoolThreads + j * nq + tid] = v;
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    s_pool[4 * tid + 0] = fmaxf(s.x + b1[4 * tid + 0], 0.f);
    s_pool[4 * tid + 1] = fmaxf(s.y + b1[4 * tid + 1], 0.f);
    s_pool[4 * tid + 2] = fmaxf(s.z + b1[4 * tid + 2], 0.f);
    s_pool[4 * tid + 3] = fmaxf(s.w + b1[4 * tid + 3], 0.f);
  }
  __syncthreads();
  if (dbg)
    for (int k = tid; k < N; k += kPoolThreads) dimg[C + k] = s_pool[k];
  {
    const int per = (N + nks - 1) / nks;
    const int k0 = min(N, ks * per), k1 = min(N, k0 + per);
    if (ks < nks) {
      const float4 r = pool_slice(w2t, s_pool, k0, k1, N, q);
      s_red[ks * nq + q] = r;
      if (dbg) dv[2 * kPoolThreads + tid] = r;
    }
  }
  __syncthreads();
  if (tid < nq) {
    float4 s = s_red[tid];
    if (dbg) dv[3 * kPoolThreads + tid] = s;
    for (int j = 1; j < nks; ++j) {
      const float4 v = s_red[j * nq + tid];
      if (dbg) dv[3 * kPoolThreads + j * nq + tid] = v;
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    *reinterpret_cast<float4*>(img_bias + (size_t)b * N + 4 * tid) = s;
  }
}

void aspp_pool(const bf16* in, float* ws, const float* w1t, const float* b1, const float* w2t,
               float* img_bias, int B, int HW, int C, int N, hipStream_t s, float* dbg, int mode) {
  if (C > kPoolMaxC || N > kPoolMaxN || C % 8 || N % 4)
    throw std::invalid_argument("aspp_pool: C <= 2048, C % 8, N <= 512, N % 4");
  if (!(mode & 2))  // bit 1 (debug): reuse the partial sums already in ws
    hipLaunchKernelGGL(gap_partial_kernel, dim3(B, kGapSlices, cdiv(C / 8, 64)), dim3(256), 0, s, in,
                       ws, HW, C);
  // mode bits 2/3 (debug): 256 / 512 threads per workgroup instead of 1024
  if (mode & 4)
    hipLaunchKernelGGL(aspp_pool_kernel<256>, dim3(B), dim3(256), 0, s, ws, w1t, b1, w2t, img_bias, HW, C,
                       N, dbg, mode);
  else if (mode & 8)
    hipLaunchKernelGGL(aspp_pool_kernel<512>, dim3(B), dim3(512), 0, s, ws, w1t, b1, w2t, img_bias, HW, C,
                       N, dbg, mode);
  else
    hipLaunchKernelGGL(aspp_pool_kernel<1024>, dim3(B), dim3(1024), 0, s, ws, w1t, b1, w2t, img_bias, HW,
                       C, N, dbg, mode);
  check_launch("aspp_pool");
}

// ---------------------------------------------------------------- upsample + argmax
// Logits of one frame (h x w x K, ~50 KB at 33x33x24 bf16) stay L1/L2 resident;
// each lane produces 4 consecutive output pixels of a row and one 4-byte store.
// Interpolation mirrors torch's upsample_bilinear2d(align_corners=True):
// src = dst * (in - 1) / (out - 1) in fp32, lerp weights (1 - l, l).
template <int KMAX>
__global__ __launch_bounds__(256) void upsample_argmax_kernel(const bf16* __restrict__ logits,
                                                              uint8_t* __restrict__ labels, int B,
                                                              int h, int w, int K, int ldk, int H,
                                                              int W) {
  const int W4 = (W + 3) / 4;
  const long long total = (long long)B * H * W4;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int xq = (int)(t % W4);
  const int Y = (int)((t / W4) % H);
  const int b = (int)(t / ((long long)W4 * H));
  const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
  const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  const float fy = sh * (float)Y;
  const int y0 = (int)fy;
  const int yp = y0 < h - 1 ? 1 : 0;
  const float ly1 = fy - (float)y0, ly0 = 1.f - ly1;
  const bf16* L = logits + (long long)b * h * w * ldk;
  uint32_t packed = 0;
  for (int e = 0; e < 4; ++e) {
    const int X = xq * 4 + e;
    if (X >= W) break;
    const float fx = sw * (float)X;
    const int x0 = (int)fx;
    const int xp = x0 < w - 1 ? 1 : 0;
    const float lx1 = fx - (float)x0, lx0 = 1.f - lx1;
    const bf16* p00 = L + ((long long)y0 * w + x0) * ldk;
    const bf16* p01 = p00 + xp * ldk;
    const bf16* p10 = p00 + (long long)yp * w * ldk;
    const bf16* p11 = p10 + xp * ldk;
    float best = -3.0e38f;
    int arg = 0;
#pragma unroll 4
    for (int k = 0; k < K; ++k) {
      const float v = ly0 * (lx0 * (float)p00[k] + lx1 * (float)p01[k]) +
                      ly1 * (lx0 * (float)p10[k] + lx1 * (float)p11[k]);
      if (v > best) { best = v; arg = k; }
    }
    packed |= (uint32_t)(arg & 0xff) << (8 * e);
  }
  uint8_t* op = labels + ((long long)b * H + Y) * W + xq * 4;
  if (xq * 4 + 3 < W && ((((uintptr_t)op) & 3) == 0)) {
    *reinterpret_cast<uint32_t*>(op) = packed;
  } else {
    for (int e = 0; e < 4 && xq * 4 + e < W; ++e) op[e] = (packed >> (8 * e)) & 0xff;
  }
}

// Separable interval variant (upsampling, K <= 32, ldk % 8 == 0): one lane = one
// output row x one source interval [j, j+1], i.e. every output pixel X of the row
// whose left source column (int)(sw * X) is j (16 of them at 33 -> 513). The lane
// vertically interpolates its two source columns once (16-byte bf16 loads) into
// fp32 registers (and their difference), after which each output pixel costs one
// FMA + compare per class: no per-pixel gathers and no register selects (PMC on
// the direct kernel: 4 x K scalar bf16 loads per pixel made it issue-bound).
// Interpolant v = v_j + lx1 * (v_{j+1} - v_j) with v_c = ly0 * L[y0][c] + ly1 * L[y1][c]:
// the same bilinear value as torch's align_corners=True in another rounding order
// (the tests check argmax agreement).
// Per-lane state of the separable interval upsample: the two vertically interpolated
// source columns j, j+1 (fp32, as v0 and dv = v1 - v0) of one output row, and the
// output pixels [xs, xe) whose left source column is j.
// wave-wide max of a per-lane int (a small loop bound made uniform)
__device__ __forceinline__ int wave_max_int(int v) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) v = max(v, __shfl_xor(v, off));
  return v;
}

// KC: the class count when the launch specialises it (PASCAL 21, Cityscapes 19), else 0
// (runtime K <= KP): the per-pixel argmax, the candidate masks and the vertical lerp then
// run over exactly KC classes instead of the padded KP = 24 (3 / 5 of 24 evaluations saved)
template <int KP, int KC = 0>
struct Interval {
  static constexpr int NK = KC ? KC : KP;  // classes the loops visit
  float v0[KP], dv[KP];
  int xs, xe;
  float sw;
  int j, w;

  __device__ void load(const bf16* __restrict__ logits, int b, int Y, int jj, int h, int ww, int H,
                       int W, int ldk) {
    j = jj;
    w = ww;
    const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
    sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
    const float fy = sh * (float)Y;
    const int y0 = (int)fy;
    const int yp = y0 < h - 1 ? 1 : 0;
    const float ly1 = fy - (float)y0, ly0 = 1.f - ly1;
    // first output column whose left source column is j (exact fp32 formula, then fix-up)
    xs = sw > 0.f ? (int)((float)j / sw) - 1 : 0;
    if (xs < 0) xs = 0;
    while (xs > 0 && (int)(sw * (float)xs) >= j) --xs;
    while (xs < W && (int)(sw * (float)xs) < j) ++xs;
    xe = xs;
    for (int e = 0; e < 32; ++e) {
      const int X = xs + e;
      if (X >= W || (int)(sw * (float)X) != j) break;
      xe = X + 1;
    }
    const int j1 = j < w - 1 ? j + 1 : j;
    const bf16* r0 = logits + ((size_t)(b * h + y0) * w) * ldk;
    const bf16* r1 = r0 + (size_t)yp * w * ldk;
#pragma unroll
    for (int k8 = 0; k8 < KP; k8 += 8) {
      const bf16x8 a0 = ld8(r0 + (size_t)j * ldk + k8), a1 = ld8(r1 + (size_t)j * ldk + k8);
      const bf16x8 c0 = ld8(r0 + (size_t)j1 * ldk + k8), c1 = ld8(r1 + (size_t)j1 * ldk + k8);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (k8 + q >= NK) continue;
        const float u = ly0 * (float)a0[q] + ly1 * (float)a1[q];
        const float v = ly0 * (float)c0[q] + ly1 * (float)c1[q];
        v0[k8 + q] = u;
        dv[k8 + q] = v - u;
      }
    }
  }

  __device__ float lx(int X) const { return j < w - 1 ? sw * (float)X - (float)j : 0.f; }

  // TAGGED: argmax as a max over index-tagged scores (the low 5 mantissa bits of each
  // score replaced by 31 - k, one v_max per class instead of a compare + two selects;
  // classes closer than 2^-18 relative may swap). Otherwise a strict-compare argmax
  // (first maximum wins, as torch.argmax). Measured on MI355X (B=32, 33->513, K=21,
  // scripts/bench_upsample.py): tagged 57.5 us vs compare 34.4 us per launch, so the
  // tagged form is kept only as a benchmarked alternative.
  template <bool TAGGED>
  __device__ int argmax_at(float lx1, int K) const {
    float best = -3.0e38f;
    int arg = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const float v = v0[k] + lx1 * dv[k];
      if (TAGGED) {
        const float t = __uint_as_float((__float_as_uint(v) & ~31u) | (unsigned)(31 - k));
        if (KC || k < K) best = fmaxf(best, t);
      } else {
        if ((KC || k < K) && v > best) { best = v; arg = k; }
      }
    }
    return TAGGED ? 31 - (int)(__float_as_uint(best) & 31u) : arg;
  }

  // Candidate pruning + class-major evaluation (variant 6). Along the interval each class
  // score is linear in lx1, so it lies between its two end values: with L the best lower
  // end, a class whose upper end is below L (minus a margin of 2^-12 of the largest end
  // magnitude, far above the interpolation's rounding) can win at no pixel of the
  // interval. A lane left with one candidate stores it; the others evaluate, pixel by pixel,
  // only the classes that are a candidate of SOME lane of the wave (their union, uniform:
  // a scalar branch skips every other class) -- class-major over NPX register-resident
  // pixels, in ascending class order with a strict compare, so the label is the first
  // maximum as in argmax_at. The per-pixel fallback of emit() evaluated all K classes at
  // up to 14 pixels of every interval whose end winners differ (2,293 VALU per wave on the
  // headline maps, r7x_headline_kernel_pmc.txt).
  template <int NPX>
  __device__ void emit_union(uint8_t* op, int K) const {
    const int n = xe - xs;
    const float t0 = lx(xs), t1 = lx(n > 0 ? xe - 1 : xs);
    float hi[KP];
    float L = -3.0e38f, M = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const float a = v0[k] + t0 * dv[k], b = v0[k] + t1 * dv[k];
      const float lo = fminf(a, b);
      hi[k] = fmaxf(a, b);
      if (KC || k < K) {
        L = fmaxf(L, lo);
        M = fmaxf(M, fmaxf(fabsf(a), fabsf(b)));
      }
    }
    const float thr = L - (M * (1.f / 4096.f) + 1e-30f);
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k)
      if ((KC || k < K) && hi[k] >= thr) m |= 1u << k;
    if (n <= 0) m = 0;
    const bool single = (m & (m - 1)) == 0;
    if (single && m) {
      const uint8_t l = (uint8_t)(__ffs(m) - 1);
      for (int X = xs; X < xe; ++X) op[X] = l;
    }
    // union over the lanes that still need per-pixel work (a wave-uniform value)
    uint32_t u = single ? 0u : m;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) u |= (uint32_t)__shfl_xor((int)u, off);
    u = __builtin_amdgcn_readfirstlane(u);
    if (u == 0) return;
    const int chunks = single ? 0 : (n + NPX - 1) / NPX;
    const int nchunk = __builtin_amdgcn_readfirstlane(wave_max_int(chunks));
    for (int c = 0; c < nchunk; ++c) {
      const int X0 = xs + c * NPX;
      float tx[NPX], best[NPX];
      int arg[NPX];
#pragma unroll
      for (int e = 0; e < NPX; ++e) {
        tx[e] = lx(X0 + e);
        best[e] = -3.0e38f;
        arg[e] = 0;
      }
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        if (u & (1u << k)) {  // uniform: a scalar branch
#pragma unroll
          for (int e = 0; e < NPX; ++e) {
            const float v = v0[k] + tx[e] * dv[k];
            if (v > best[e]) { best[e] = v; arg[e] = k; }
          }
        }
      }
      if (c < chunks) {
#pragma unroll
        for (int e = 0; e < NPX; ++e)
          if (X0 + e < xe) op[X0 + e] = (uint8_t)arg[e];
      }
    }
  }

  // Per-lane candidates (variant 7): the candidate mask as in emit_union, then each lane
  // evaluates ITS OWN candidates only. Registers cannot be indexed by a lane-varying class,
  // so the lane's (v0, dv) pairs go to a private LDS column first ([class][lane] float2:
  // every read conflict-free whatever the classes) and the candidate loop reads them back
  // by class. A wave runs max over its lanes of the candidate count (compact 16-row x
  // 4-interval waves keep the counts alike), instead of the union's class count.
  template <int NPX>
  __device__ void emit_cand(uint8_t* op, int K, float2* col) const {
    const int n = xe - xs;
    const float t0 = lx(xs), t1 = lx(n > 0 ? xe - 1 : xs);
    float hi[KP];
    float L = -3.0e38f, M = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const float a = v0[k] + t0 * dv[k], b = v0[k] + t1 * dv[k];
      const float lo = fminf(a, b);
      hi[k] = fmaxf(a, b);
      if (KC || k < K) {
        L = fmaxf(L, lo);
        M = fmaxf(M, fmaxf(fabsf(a), fabsf(b)));
      }
    }
    const float thr = L - (M * (1.f / 4096.f) + 1e-30f);
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k)
      if ((KC || k < K) && hi[k] >= thr) m |= 1u << k;
    if (n <= 0) return;
    if ((m & (m - 1)) == 0) {
      const uint8_t l = (uint8_t)(__ffs(m) - 1);
      for (int X = xs; X < xe; ++X) op[X] = l;
      return;
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) col[k * 256] = make_float2(v0[k], dv[k]);
    for (int X0 = xs; X0 < xe; X0 += NPX) {
      float tx[NPX], best[NPX];
      int arg[NPX];
#pragma unroll
      for (int e = 0; e < NPX; ++e) {
        tx[e] = lx(X0 + e);
        best[e] = -3.0e38f;
        arg[e] = 0;
      }
      uint32_t mm = m;
      while (mm) {  // ascending class order, strict compare: the first maximum wins
        const int k = __ffs(mm) - 1;
        mm &= mm - 1;
        const float2 c = col[k * 256];
#pragma unroll
        for (int e = 0; e < NPX; ++e) {
          const float v = c.x + tx[e] * c.y;
          if (v > best[e]) { best[e] = v; arg[e] = k; }
        }
      }
#pragma unroll
      for (int e = 0; e < NPX; ++e)
        if (X0 + e < xe) op[X0 + e] = (uint8_t)arg[e];
    }
  }

  // Along the interval every class score is LINEAR in lx1, and the max of linear
  // functions is convex: when one class wins at both end pixels it wins at every
  // pixel in between. The common case (smooth logits) then costs two argmaxes
  // instead of one per pixel (up to 16).
  template <bool TAGGED>
  __device__ void emit(uint8_t* op, int K) const {
    if (xe == xs) return;
    const int a0 = argmax_at<TAGGED>(lx(xs), K);
    const int a1 = xe - 1 > xs ? argmax_at<TAGGED>(lx(xe - 1), K) : a0;
    if (a0 == a1) {
      for (int X = xs; X < xe; ++X) op[X] = (uint8_t)a0;
      return;
    }
    op[xs] = (uint8_t)a0;
    op[xe - 1] = (uint8_t)a1;
    for (int X = xs + 1; X < xe - 1; ++X) op[X] = (uint8_t)argmax_at<TAGGED>(lx(X), K);
  }
};

// Separable interval variant (upsampling, K <= 32, ldk % 8 == 0): one lane = one
// output row x one source interval [j, j+1], i.e. every output pixel X of the row
// whose left source column (int)(sw * X) is j (16 of them at 33 -> 513). The lane
// vertically interpolates its two source columns once (16-byte bf16 loads) into
// fp32 registers (and their difference), after which each output pixel costs one
// FMA + compare per class: no per-pixel gathers and no register selects (PMC on
// the direct kernel: 4 x K scalar bf16 loads per pixel made it issue-bound).
// Interpolant v = v_j + lx1 * (v_{j+1} - v_j) with v_c = ly0 * L[y0][c] + ly1 * L[y1][c]:
// the same bilinear value as torch's align_corners=True in another rounding order
// (the tests check argmax agreement). Labels are stored straight from the lane: up to
// 16 byte stores per lane, 16 bytes apart across the wave.
template <int KP, int KC, bool TAGGED>
__global__ __launch_bounds__(256) void upsample_argmax_interval_kernel(
    const bf16* __restrict__ logits, uint8_t* __restrict__ labels, int B, int h, int w, int K,
    int ldk, int H, int W) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * H * w) return;
  const int j = t % w;
  const int Y = (t / w) % H;
  const int b = t / (w * H);
  Interval<KP, KC> iv;
  iv.load(logits, b, Y, j, h, w, H, W, ldk);
  iv.template emit<TAGGED>(labels + ((size_t)b * H + Y) * W, K);
}

// variant 6: emit_union. A wave owns a compact 16-row x 4-interval block (lane = row dy +
// 16 x interval dj): at 33 -> 513 its 16 rows share one upper source row, so the wave's
// union of candidate classes is that of ~4 source cells, not of a whole map row as with
// the row-major lane order. The wave-wide shuffles need every lane: lanes past the map
// take an empty interval instead of returning.
template <int KP, int KC>
__global__ __launch_bounds__(256) void upsample_argmax_union_kernel(
    const bf16* __restrict__ logits, uint8_t* __restrict__ labels, int B, int h, int w, int K,
    int ldk, int H, int W) {
  const int nyb = (H + 15) >> 4, njb = (w + 3) >> 2;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int jb = wave % njb, yb = (wave / njb) % nyb, b0 = wave / (njb * nyb);
  const int Y0 = yb * 16 + (lane & 15), j0 = jb * 4 + (lane >> 4);
  const bool live = b0 < B && Y0 < H && j0 < w;
  const int b = live ? b0 : 0, Y = live ? Y0 : 0, j = live ? j0 : 0;
  Interval<KP, KC> iv;
  iv.load(logits, b, Y, j, h, w, H, W, ldk);
  if (!live) iv.xe = iv.xs;
  iv.template emit_union<16>(labels + ((size_t)b * H + Y) * W, K);
}

// variant 7: emit_cand on the union kernel's compact waves; a lane's private LDS column
// holds its (v0, dv) pairs (KP x 8 B per lane: 48 KiB per 256-lane workgroup at KP = 24)
template <int KP, int KC>
__global__ __launch_bounds__(256) void upsample_argmax_cand_kernel(
    const bf16* __restrict__ logits, uint8_t* __restrict__ labels, int B, int h, int w, int K,
    int ldk, int H, int W) {
  __shared__ float2 cols[KP * 256];
  const int nyb = (H + 15) >> 4, njb = (w + 3) >> 2;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int jb = wave % njb, yb = (wave / njb) % nyb, b = wave / (njb * nyb);
  const int Y = yb * 16 + (lane & 15), j = jb * 4 + (lane >> 4);
  if (b >= B || Y >= H || j >= w) return;  // no wave-wide operation below
  Interval<KP, KC> iv;
  iv.load(logits, b, Y, j, h, w, H, W, ldk);
  iv.template emit_cand<16>(labels + ((size_t)b * H + Y) * W, K, cols + threadIdx.x);
}

// Row-block variant: a workgroup owns R = 256 / w whole output rows (consecutive in the
// B*H row space, so one contiguous R*W-byte run of the label buffer). Each lane
// computes one interval as above into an LDS copy of the rows; the workgroup then
// writes the run with coalesced dword stores (byte stores only for the unaligned head
// and tail) instead of 16 scattered byte stores per lane. Measured on MI355X: 38.9 us
// vs 34.4 us for the per-lane stores (the kernel is not store-bound; the 7-row blocks
// leave 25 of 256 lanes idle and add a barrier), so the plan autotuner picks between
// the two per shape.
template <int KP, int KC, bool TAGGED>
__global__ __launch_bounds__(256) void upsample_argmax_rows_kernel(
    const bf16* __restrict__ logits, uint8_t* __restrict__ labels, int B, int h, int w, int K,
    int ldk, int H, int W, int R) {
  extern __shared__ uint8_t rows_lds[];
  const int tid = threadIdx.x;
  const long long g0 = (long long)blockIdx.x * R;  // first global row (b * H + Y)
  const long long nrows = (long long)B * H;
  const int nr = (int)(nrows - g0 < R ? nrows - g0 : R);
  const int r = tid / w, j = tid % w;
  if (r < nr) {
    const long long g = g0 + r;
    Interval<KP, KC> iv;
    iv.load(logits, (int)(g / H), (int)(g % H), j, h, w, H, W, ldk);
    iv.template emit<TAGGED>(rows_lds + r * W, K);
  }
  __syncthreads();
  const int n = nr * W;
  uint8_t* out = labels + g0 * W;
  const int head = (int)((4 - ((uintptr_t)out & 3)) & 3) < n ? (int)((4 - ((uintptr_t)out & 3)) & 3) : n;
  if (tid < head) out[tid] = rows_lds[tid];
  const int nd = (n - head) >> 2;
  uint32_t* outd = reinterpret_cast<uint32_t*>(out + head);
  for (int i = tid; i < nd; i += 256) {
    const uint8_t* q = rows_lds + head + 4 * i;
    outd[i] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
  }
  const int tail0 = head + 4 * nd;
  if (tid < n - tail0) out[tail0 + tid] = rows_lds[tail0 + tid];
}

namespace {

template <int KP, int KC>
void launch_upsample_interval(int variant, const bf16* logits, uint8_t* labels, int B, int h,
                              int w, int K, int ldk, int H, int W, hipStream_t s) {
  const long long total = (long long)B * H * w;
  if (variant == 6 || variant == 7) {
    const long long waves = (long long)B * ((H + 15) / 16) * ((w + 3) / 4);
    if (variant == 6)
      hipLaunchKernelGGL((upsample_argmax_union_kernel<KP, KC>), dim3(cdiv(waves, 4)), dim3(256), 0, s,
                         logits, labels, B, h, w, K, ldk, H, W);
    else
      hipLaunchKernelGGL((upsample_argmax_cand_kernel<KP, KC>), dim3(cdiv(waves, 4)), dim3(256), 0, s,
                         logits, labels, B, h, w, K, ldk, H, W);
    return;
  }
  if (variant == 1 || variant == 2) {
    if (variant == 1)
      hipLaunchKernelGGL((upsample_argmax_interval_kernel<KP, KC, false>), dim3(cdiv(total, 256)),
                         dim3(256), 0, s, logits, labels, B, h, w, K, ldk, H, W);
    else
      hipLaunchKernelGGL((upsample_argmax_interval_kernel<KP, KC, true>), dim3(cdiv(total, 256)),
                         dim3(256), 0, s, logits, labels, B, h, w, K, ldk, H, W);
    return;
  }
  const int R = 256 / w;
  const long long nrows = (long long)B * H;
  const size_t lds = (size_t)R * W;
  if (variant == 3)
    hipLaunchKernelGGL((upsample_argmax_rows_kernel<KP, KC, false>), dim3(cdiv(nrows, R)), dim3(256),
                       lds, s, logits, labels, B, h, w, K, ldk, H, W, R);
  else
    hipLaunchKernelGGL((upsample_argmax_rows_kernel<KP, KC, true>), dim3(cdiv(nrows, R)), dim3(256),
                       lds, s, logits, labels, B, h, w, K, ldk, H, W, R);
}

}  // namespace

// variant: 0 = default (per-lane interval, strict-compare argmax), 1 = interval / compare,
// 2 = interval / tagged max, 3 = row-block / compare, 4 = row-block / tagged max,
// 5 = the direct (per-pixel gather) kernel, 6 = interval / wave-union candidates,
// 7 = interval / per-lane candidates. Variants 1-4, 6 and 7 need the interval
// preconditions; otherwise the direct kernel runs.
void upsample_argmax(const bf16* logits, uint8_t* labels, int B, int h, int w, int K, int ldk,
                     int H, int W, hipStream_t s, int variant) {
  if (K > 256) throw std::invalid_argument("upsample_argmax: K > 256");
  if (variant < 0 || variant > 7) throw std::invalid_argument("upsample_argmax: bad variant");
  if (variant == 0) variant = 1;
  // interval path: at most 32 output pixels share a left source column; the row-block
  // variant needs a whole row of intervals in one workgroup and R * W bytes of LDS
  const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  const bool interval = K <= 32 && ldk % 8 == 0 && ldk >= ((K + 7) / 8) * 8 && w >= 2 && W > 1 &&
                        sw > 0.f && 1.f / sw <= 30.f && (long long)B * H * w < (1LL << 31);
  if (interval && (variant == 3 || variant == 4) && (w > 256 || (256 / w) * W > 65536))
    variant -= 2;
  if (interval && variant != 5) {
    // exact class counts of the shipped label sets (PASCAL VOC 21, Cityscapes 19)
    if (K == 21)
      launch_upsample_interval<24, 21>(variant, logits, labels, B, h, w, K, ldk, H, W, s);
    else if (K == 19)
      launch_upsample_interval<24, 19>(variant, logits, labels, B, h, w, K, ldk, H, W, s);
    else if (K <= 24)
      launch_upsample_interval<24, 0>(variant, logits, labels, B, h, w, K, ldk, H, W, s);
    else
      launch_upsample_interval<32, 0>(variant, logits, labels, B, h, w, K, ldk, H, W, s);
    check_launch("upsample_argmax interval");
    return;
  }
  const long long total = (long long)B * H * ((W + 3) / 4);
  hipLaunchKernelGGL(upsample_argmax_kernel<256>, dim3(cdiv(total, 256)), dim3(256), 0, s, logits,
                     labels, B, h, w, K, ldk, H, W);
  check_launch("upsample_argmax");
}

}  // namespace ssa
