// Implicit-GEMM convolution on MFMA (gfx950), NHWC bf16 in/out, fp32 accumulate.
//
//   out[b, oy, ox, co_off + n] = act( sum_{ky,kx,c} W[n][ky][kx][c] * in[b, iy, ix, c]
//                                     + bias[n] + img_bias[b][n] + res[b, oy, ox, n] )
//   iy = oy*stride + (ky - KH/2)*dil, ix = ox*stride + (kx - KW/2)*dil, zero outside.
//
// Covers every dense conv of the models: MobileNetV2 1x1 expand/project (fused
// residual), ASPP 1x1 / 3x3 atrous branches (written straight into their channel
// slice of the concat buffer: concat-free), the ASPP projection (the image-pool
// branch enters as a per-image bias), the logits layer, and the ResNet-50
// bottleneck 1x1/3x3 (strided) convs.
//
// Mapping: the MFMA's A operand is the weight tile (rows = output channels) and
// the B operand is the pixel tile, so each lane's accumulator holds 4 consecutive
// output channels of one pixel (v_mfma_f32_16x16x32_bf16 C/D layout: row =
// (lane>>4)*4 + r, col = lane&15) and the epilogue stores 8 contiguous bytes.
// Both operands are 16-byte vector loads straight to VGPRs in the MFMA fragment
// layout (lane l: 8 consecutive K elements at k = 8*(l>>4), row/col l&15); taps
// that fall entirely outside the image for all of a wave's pixels are skipped
// (wave-uniform), which removes most of the zero work of the rate-12/18 ASPP
// branches on a 33x33 map.
//
// Block: 4 waves in a 2x2 arrangement; wave tile = (16*MT pixels) x (16*NT chans).
#include "common.h"
#include "kernels.h"

namespace ssa {

struct ConvArgs {
  const bf16* in; const bf16* w; const float* bias; const float* img_bias;
  const bf16* res; bf16* out;
  int B, IH, IW, Cin, OH, OW, Cout;
  int KH, KW, stride, dil;
  int ldo, co_off, ldr, act;
};

template <int MT, int NT>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = a.B * a.OH * a.OW;
  const int tiles_m = cdiv_dev(M, 32 * MT);
  const int tiles_n = cdiv_dev(a.Cout, 32 * NT);
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  const int pix0 = tm * 32 * MT + wm * 16 * MT;
  const int ch0 = tn * 32 * NT + wn * 16 * NT;
  const int r = lane & 15, kq = lane >> 4;  // fragment row/col and K quarter

  // per-subtile pixel coordinates for this lane's B-fragment column
  int pb[MT], py[MT], px[MT];
  bool pvalid[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = pix0 + i * 16 + r;
    pvalid[i] = m < M;
    const int mm = pvalid[i] ? m : 0;
    pb[i] = mm / (a.OH * a.OW);
    const int rem = mm - pb[i] * a.OH * a.OW;
    py[i] = (rem / a.OW) * a.stride;
    px[i] = (rem % a.OW) * a.stride;
  }
  // weight rows for this lane's A-fragment
  bool wvalid[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wvalid[j] = (ch0 + j * 16 + r) < a.Cout;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int taps = a.KH * a.KW;
  const long long wrow = (long long)taps * a.Cin;  // weight elements per out channel
  for (int t = 0; t < taps; ++t) {
    const int dy = (t / a.KW - a.KH / 2) * a.dil;
    const int dx = (t % a.KW - a.KW / 2) * a.dil;
    long long off[MT];
    bool ok[MT];
    bool any = false;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int iy = py[i] + dy, ix = px[i] + dx;
      ok[i] = pvalid[i] && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
      off[i] = (((long long)pb[i] * a.IH + iy) * a.IW + ix) * a.Cin;
      any |= ok[i];
    }
    if (!__any(any)) continue;  // wave-uniform skip of an all-padding tap
    const bf16* wt = a.w + (long long)t * a.Cin;
    for (int c0 = 0; c0 < a.Cin; c0 += 32) {
      const int c = c0 + kq * 8;
      const bool cok = c < a.Cin;
      bf16x8 bfr[MT], afr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        bfr[i] = (ok[i] && cok) ? ld8(a.in + off[i] + c) : zero8();
#pragma unroll
      for (int j = 0; j < NT; ++j)
        afr[j] = (wvalid[j] && cok) ? ld8(wt + (long long)(ch0 + j * 16 + r) * wrow + c) : zero8();
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[j], bfr[i], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: lane holds out channels ch0 + j*16 + kq*4 + {0..3} of pixel pix0 + i*16 + r
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = pix0 + i * 16 + r;
    if (m >= M) continue;
    const int b = pb[i];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = ch0 + j * 16 + kq * 4;
      if (n >= a.Cout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      const bool full = n + 3 < a.Cout;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (n + q < a.Cout) {
          v[q] += a.bias[n + q];
          if (a.img_bias) v[q] += a.img_bias[(long long)b * a.Cout + n + q];
        }
      }
      if (a.res) {
        const bf16* rp = a.res + (long long)m * a.ldr + n;
        if (full && (a.ldr & 3) == 0) {
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(rp);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += (float)rv[q];
        } else {
          for (int q = 0; q < 4; ++q) if (n + q < a.Cout) v[q] += (float)rp[q];
        }
      }
      bf16* op = a.out + (long long)m * a.ldo + a.co_off + n;
      if (full && ((a.ldo | a.co_off) & 3) == 0) {
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)apply_act(v[q], a.act);
        *reinterpret_cast<bf16x4*>(op) = o;
      } else {
        for (int q = 0; q < 4; ++q)
          if (n + q < a.Cout) op[q] = (bf16)apply_act(v[q], a.act);
      }
    }
  }
}

template <int MT, int NT>
static void launch_conv(const ConvArgs& a, hipStream_t s) {
  const int M = a.B * a.OH * a.OW;
  const int grid = cdiv(M, 32 * MT) * cdiv(a.Cout, 32 * NT);
  hipLaunchKernelGGL((conv_gemm_kernel<MT, NT>), dim3(grid), dim3(256), 0, s, a);
  check_launch("conv_gemm");
}

void conv_gemm(const ConvParams& p, hipStream_t s) {
  if (p.Cin % 8 != 0) throw std::invalid_argument("conv_gemm: Cin must be a multiple of 8");
  if (p.co_off % 1 != 0 || p.ldo < p.co_off + p.Cout) throw std::invalid_argument("conv_gemm: bad ldo/co_off");
  if (p.res && p.ldr < p.Cout) throw std::invalid_argument("conv_gemm: bad ldr");
  ConvArgs a{p.in, p.w, p.bias, p.img_bias, p.res, p.out, p.B, p.IH, p.IW, p.Cin, p.OH, p.OW,
             p.Cout, p.KH, p.KW, p.stride, p.dil, p.ldo, p.co_off, p.ldr, p.act};
  const long long M = (long long)p.B * p.OH * p.OW;
  // tile choice: wide channel tiles for wide outputs, narrow for the thin ones
  if (p.Cout <= 32) {
    launch_conv<4, 1>(a, s);  // 128 px x 32 ch
  } else if (p.Cout <= 64 || M < 8192) {
    launch_conv<2, 2>(a, s);  // 64 px x 64 ch
  } else {
    launch_conv<2, 4>(a, s);  // 64 px x 128 ch
  }
}

}  // namespace ssa
