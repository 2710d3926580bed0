// Minimal standalone reproducer for the round-3 finding (profiles/r3_packed_f32_race.txt):
// packed-f32 VALU results (v_pk_fma_f32) came back wrong in the low halves of lanes 48-63
// when waves of MFMA-heavy kernels shared the SIMD. Two kernels, no framework:
//
//   pk_dot      every thread accumulates float2 partial dot products over a strided
//               input (the shape of aspp_pool's GAP x W partials, where the corruption
//               was caught), written out per thread;
//   mfma_noise  back-to-back v_mfma_f32_32x32x16_bf16 on register operands, launched on
//               two other streams so its waves are co-resident with pk_dot's.
//
// pk_dot is first run alone (reference); then REPS times concurrently with the noise, and
// every thread's result is compared bit for bit. Build twice (the flag is the one the
// extension is built with, ops/build.py):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 csrc/tools/packed_f32_repro.hip -o repro_pk
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Xclang -target-feature -Xclang -packed-fp32-ops \
//         csrc/tools/packed_f32_repro.hip -o repro_nopk
//   ./repro_pk [reps]; ./repro_nopk [reps]
// Expected if the finding holds: mismatches with repro_pk, none with repro_nopk. The
// program prints the counts and the lane histogram; it exits 0 either way (a measurement).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

static void chk(hipError_t e, const char* w) {
  if (e != hipSuccess) {
    fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e));
    exit(1);
  }
}

// out[t] = sum_k x[k * ld + c] * w[k * N + n] for 4 consecutive n per thread, accumulated
// as two float2 pairs (the compiler emits v_pk_fma_f32 when packed-f32 ops are enabled)
__global__ __launch_bounds__(1024) void pk_dot(const float* __restrict__ x, const float* __restrict__ w,
                                               float* __restrict__ out, int K, int N) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int n0 = (t * 4) % N;
  const float* xr = x + (t % 320);
  f32x2 a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
  for (int k = 0; k < K; ++k) {
    const float xv = xr[k * 320];
    const f32x4 wv = *reinterpret_cast<const f32x4*>(w + (size_t)k * N + n0);
    const f32x2 xx = {xv, xv};
    a0 = __builtin_elementwise_fma(xx, f32x2{wv.x, wv.y}, a0);
    a1 = __builtin_elementwise_fma(xx, f32x2{wv.z, wv.w}, a1);
  }
  *reinterpret_cast<f32x4*>(out + (size_t)t * 4) = f32x4{a0.x, a0.y, a1.x, a1.y};
}

__global__ __launch_bounds__(256) void mfma_noise(float* __restrict__ sink, int iters, float seed) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(seed + 0.001f * (threadIdx.x + i));
    b[i] = (__bf16)(seed - 0.002f * (threadIdx.x + i));
  }
  f32x16 acc0 = {}, acc1 = {};
  for (int i = 0; i < iters; ++i) {
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc1, 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += acc0[i] - acc1[i];
  if (s == 12345.f) sink[threadIdx.x] = s;  // never true; keeps the loop
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 400;
  const int K = 1089, N = 256, C = 320;
  const int threads = 1024, blocks = 64;  // 64 x 1024 threads, 4 outputs each
  const int nout = threads * blocks * 4;
  std::vector<float> hx((size_t)K * C), hw((size_t)K * N);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 65536.f - 0.5f; };
  for (auto& v : hx) v = rnd();
  for (auto& v : hw) v = rnd();
  float *x, *w, *out, *sink;
  chk(hipMalloc(&x, hx.size() * 4), "malloc");
  chk(hipMalloc(&w, hw.size() * 4), "malloc");
  chk(hipMalloc(&out, (size_t)nout * 4), "malloc");
  chk(hipMalloc(&sink, 4096), "malloc");
  chk(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice), "h2d");
  chk(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice), "h2d");
  hipStream_t st[3];
  for (auto& q : st) chk(hipStreamCreateWithFlags(&q, hipStreamNonBlocking), "stream");
  hipLaunchKernelGGL(pk_dot, dim3(blocks), dim3(threads), 0, st[0], x, w, out, K, N);
  chk(hipDeviceSynchronize(), "ref");
  std::vector<float> ref(nout), got(nout);
  chk(hipMemcpy(ref.data(), out, (size_t)nout * 4, hipMemcpyDeviceToHost), "d2h");
  long bad_runs = 0, bad_vals = 0;
  long lane_hist[64] = {0}, half_hist[2] = {0};
  for (int r = 0; r < reps; ++r) {
    chk(hipMemsetAsync(out, 0, (size_t)nout * 4, st[0]), "memset");
    hipLaunchKernelGGL(mfma_noise, dim3(512), dim3(256), 0, st[1], sink, 4000, 0.5f + r * 1e-3f);
    hipLaunchKernelGGL(mfma_noise, dim3(512), dim3(256), 0, st[2], sink, 4000, 0.25f + r * 1e-3f);
    for (int j = 0; j < 8; ++j)
      hipLaunchKernelGGL(pk_dot, dim3(blocks), dim3(threads), 0, st[0], x, w, out, K, N);
    chk(hipDeviceSynchronize(), "run");
    chk(hipMemcpy(got.data(), out, (size_t)nout * 4, hipMemcpyDeviceToHost), "d2h");
    long b = 0;
    for (int i = 0; i < nout; ++i)
      if (memcmp(&got[i], &ref[i], 4) != 0) {
        ++b;
        const int t = i / 4;
        ++lane_hist[t % 64];
        ++half_hist[(i % 4) & 1];  // 0: low half of a packed pair (x / z), 1: high half
      }
    bad_vals += b;
    bad_runs += b != 0;
  }
  printf("packed_f32_repro: %s build, %d runs (8 pk_dot launches each beside 2 MFMA noise kernels)\n",
#if defined(__AMDGCN__)
         "device",
#else
         "host",
#endif
         reps);
  printf("mismatching runs %ld / %d, mismatching values %ld (low halves %ld, high halves %ld)\n",
         bad_runs, reps, bad_vals, half_hist[0], half_hist[1]);
  if (bad_vals) {
    printf("lane histogram (lane: count):");
    for (int l = 0; l < 64; ++l)
      if (lane_hist[l]) printf(" %d:%ld", l, lane_hist[l]);
    printf("\n");
  }
  return 0;
}
