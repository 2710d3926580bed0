// Shared helpers for the gfx950 (CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

namespace ssa {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

constexpr int kWave = 64;

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_RELU6 = 2 };

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  if (act == ACT_RELU6) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

// 16-byte vector load/store of 8 bf16.
__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
// 16 bytes at a uniform base + a 32-bit BYTE offset: the zero-extended 32-bit offset is
// what lets the compiler pick the SGPR-base + VGPR-offset global addressing form (an
// element offset is scaled in 64 bits and costs a 64-bit VALU add per access)
__device__ __forceinline__ bf16x8 ld8_at(const bf16* base, unsigned byte_off) {
  return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(base) + byte_off);
}
__device__ __forceinline__ void st8(bf16* p, bf16x8 v) { *reinterpret_cast<bf16x8*>(p) = v; }

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}

// Bijective XCD-aware remap of a linear block id: blocks b and b+8 land on the
// same XCD under round-robin dispatch, so give each XCD a contiguous chunk of
// the logical tile space (speed only, never correctness).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int nx = 8;
  if (nblocks < nx * 2) return bid;
  const int q = nblocks / nx, r = nblocks % nx;
  const int xcd = bid % nx, idx = bid / nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__host__ __device__ __forceinline__ int cdiv_dev(int a, int b) { return (a + b - 1) / b; }

// Taps (bit ky * KW + kx) of a KH x KW 'same' conv whose input pixel is inside the image for
// the output pixel at input position (ay, ax): separable in y and x, so O(KH + KW) compares
// and no per-tap division (the per-tap t / KW, t % KW form was ~40 VALU per tap per row in
// the LDS-DMA GEMM prologues: a visible share of a short-K tile's VALU stream)
__device__ __forceinline__ int conv_tap_mask(int ay, int ax, int KH, int KW, int dil, int IH, int IW) {
  int xb = 0;
  for (int kx = 0; kx < KW; ++kx) {
    const int ix = ax + (kx - KW / 2) * dil;
    xb |= (ix >= 0 && ix < IW ? 1 : 0) << kx;
  }
  int bits = 0;
  for (int ky = 0; ky < KH; ++ky) {
    const int iy = ay + (ky - KH / 2) * dil;
    if (iy >= 0 && iy < IH) bits |= xb << (ky * KW);
  }
  return bits;
}

// Letterboxed camera pixels of an IHT x IWT model-input window at (iy0, ix0) ->
// LDS as normalised bf16 RGB0 (x / 127.5 - 1, BGR -> RGB; -1 for letterbox
// padding, 0 outside the H x W model input = conv zero padding). Model pixel
// (y, x) is camera pixel (lut_y[y], lut_x[x]), -1 = padding. Each pixel is a
// dependent chain (LUT load -> pixel load) and the stems are latency-bound here,
// so every lane batches GU pixels: all LUT loads, then all pixel loads, then all
// LDS stores (GU chains in flight instead of one).
template <int GU, int NT>
__device__ __forceinline__ void gather_letterbox_rgb0(bf16* IN, const uint8_t* fb, const int32_t* lut_x,
                                                      const int32_t* lut_y, int Wc, int H, int W, int iy0,
                                                      int ix0, int IHT, int IWT, int tid) {
  const int n_in = IHT * IWT;
  const float inv_iwt = 1.f / IWT;
  for (int i0 = tid; i0 < n_in; i0 += NT * GU) {
    int sidx[GU];  // >= 0: camera byte offset; -1: letterbox padding; -2: conv zero padding
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int i = i0 + u * NT;
      const int ry = (int)(((float)i + 0.5f) * inv_iwt);  // i / IWT (i < 2^14)
      const int y = iy0 + ry, x = ix0 + (i - ry * IWT);
      sidx[u] = -2;
      if (i < n_in && y >= 0 && y < H && x >= 0 && x < W) {
        const int sy = lut_y[y], sx = lut_x[x];
        sidx[u] = (sy >= 0 && sx >= 0) ? (sy * Wc + sx) * 3 : -1;
      }
    }
    uint8_t pb[GU][3];
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const uint8_t* px = fb + (sidx[u] >= 0 ? sidx[u] : 0);
      pb[u][0] = px[0]; pb[u][1] = px[1]; pb[u][2] = px[2];
    }
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int i = i0 + u * NT;
      if (i >= n_in) break;
      float rgb[3] = {0.f, 0.f, 0.f};
      if (sidx[u] >= 0) {
        rgb[0] = pb[u][2] * (1.f / 127.5f) - 1.f;
        rgb[1] = pb[u][1] * (1.f / 127.5f) - 1.f;
        rgb[2] = pb[u][0] * (1.f / 127.5f) - 1.f;
      } else if (sidx[u] == -1) {
        rgb[0] = rgb[1] = rgb[2] = -1.f;
      }
      const bf16x4 v = {(bf16)rgb[0], (bf16)rgb[1], (bf16)rgb[2], (bf16)0.f};
      *reinterpret_cast<bf16x4*>(IN + (size_t)i * 4) = v;
    }
  }
}

inline void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

inline void check_launch(const char* what) { check(hipGetLastError(), what); }

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace ssa
