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

inline void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

inline void check_launch(const char* what) { check(hipGetLastError(), what); }

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace ssa
