// Standalone timing harness for the device post-processing (postprocess.hip), built
// against one copy of that file so two versions can be A/B-timed (and kernel-traced
// with rocprofv3) on identical label maps without the Python stack:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/hip csrc/tools/post_bench.hip \
//         csrc/hip/postprocess.hip -o post_bench
//   ./post_bench [reps] [maps.bin [only]]      (SSA_POST_ACCUM=0|1 env: strips / tiles pass)
// (maps.bin: raw [32, 513, 513] uint8 label maps, e.g. the bench model's output dumped by
// scripts/label_stats.py, timed as a fourth kind "file")
// Maps: B = 32 frames of 513 x 513 cropped to 513 x 385 (the headline's 640x480
// letterbox). "flat": background and a non-masked class; "planted": 3-10 ellipses of
// person / car per frame, some with holes and islands; "noisy": planted + 1 % salt.
#include "kernels.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using namespace ssa;

static void chk(hipError_t e, const char* w) {
  if (e != hipSuccess) {
    fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e));
    exit(1);
  }
}

static void pascal(std::vector<int32_t>& pal) {
  pal.assign(256 * 3, 0);
  for (int i = 0; i < 256; ++i) {
    int c = i, r = 0, g = 0, b = 0;
    for (int s = 7; s >= 0; --s) {
      r |= ((c >> 0) & 1) << s;
      g |= ((c >> 1) & 1) << s;
      b |= ((c >> 2) & 1) << s;
      c >>= 3;
    }
    pal[i * 3] = r; pal[i * 3 + 1] = g; pal[i * 3 + 2] = b;
  }
}

static void make_maps(std::vector<uint8_t>& m, int B, int H, int W, int ch, int cw, int kind, unsigned seed) {
  std::mt19937 rng(seed);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  m.assign((size_t)B * H * W, 0);
  for (int b = 0; b < B; ++b) {
    uint8_t* f = m.data() + (size_t)b * H * W;
    if (kind == 0) {
      for (int y = 0; y < ch; ++y)
        for (int x = 200; x < cw; ++x) f[y * W + x] = 12;
      continue;
    }
    if (kind == 4) {  // lattice: 3x3 person blocks at period 4 -> one fg pixel each after the
                      // blur, ~12k components per frame: past the LDS merge's caps (fallback)
      for (int y = 0; y < ch; ++y)
        for (int x = 0; x < cw; ++x) f[y * W + x] = (y % 4 < 3 && x % 4 < 3) ? 15 : 0;
      continue;
    }
    const int nb = 3 + (int)(U(rng) * 8);
    for (int k = 0; k < nb; ++k) {
      const float cx = U(rng) * cw, cy = U(rng) * ch, rx = 10 + U(rng) * 90, ry = 10 + U(rng) * 90;
      const uint8_t cls = U(rng) < 0.5f ? 15 : 7;
      const bool hole = U(rng) < 0.3f;
      for (int y = 0; y < ch; ++y)
        for (int x = 0; x < cw; ++x) {
          const float dx = (x - cx) / rx, dy = (y - cy) / ry, d = dx * dx + dy * dy;
          if (d < 1.f) f[y * W + x] = (hole && d < 0.2f) ? (d < 0.05f ? 7 : 0) : cls;
        }
    }
    if (kind == 2)
      for (int y = 0; y < ch; ++y)
        for (int x = 0; x < cw; ++x)
          if (U(rng) < 0.01f) f[y * W + x] = U(rng) < 0.5f ? 15 : 0;
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const int B = 32, H = 513, W = 513, ch = 385, cw = 513, K = 64, bins = 32;
  std::vector<int32_t> pal;
  pascal(pal);
  int32_t* dpal;
  uint8_t* dlab;
  float* drec;
  void* ws;
  const size_t wsb = post_workspace_bytes(B, H, W, K, bins);
  chk(hipMalloc(&dpal, pal.size() * 4), "malloc pal");
  chk(hipMalloc(&dlab, (size_t)B * H * W), "malloc lab");
  chk(hipMalloc(&drec, (size_t)B * (1 + 5 * K) * 4), "malloc rec");
  chk(hipMalloc(&ws, wsb), "malloc ws");
  chk(hipMemset(ws, 0, wsb), "memset ws");
  chk(hipMemcpy(dpal, pal.data(), pal.size() * 4, hipMemcpyHostToDevice), "pal");
  hipStream_t s;
  chk(hipStreamCreate(&s), "stream");
  hipEvent_t e0, e1;
  chk(hipEventCreate(&e0), "ev");
  chk(hipEventCreate(&e1), "ev");
  printf("workspace %.1f MB/frame\n", wsb / (double)B / 1e6);
  const char* names[5] = {"flat", "planted", "noisy", "file", "lattice"};
  // kinds 0-2 and 4 (lattice: the union-find fallback); 3 = argv[2]'s maps (argv[3]: only those)
  std::vector<int> kinds = {0, 1, 2, 4};
  if (argc > 2) kinds.push_back(3);
  if (argc > 3) kinds = {3};
  std::vector<float> rec((size_t)B * (1 + 5 * K));
  for (int kind : kinds) {
    std::vector<uint8_t> maps;
    if (kind != 3) {
      make_maps(maps, B, H, W, ch, cw, kind, 1234 + kind);
    } else {
      maps.resize((size_t)B * H * W);
      FILE* fp = fopen(argv[2], "rb");
      if (!fp || fread(maps.data(), 1, maps.size(), fp) != maps.size()) {
        fprintf(stderr, "cannot read %s\n", argv[2]);
        return 1;
      }
      fclose(fp);
    }
    chk(hipMemcpy(dlab, maps.data(), maps.size(), hipMemcpyHostToDevice), "lab");
    PostParams p;
    p.labels = dlab; p.B = B; p.H = H; p.W = W; p.crop_h = ch; p.crop_w = cw;
    p.palette = dpal; p.thr = 127; p.min_area = 0.002 * H * W; p.num_bins = bins; p.K = K;
    p.ws = ws; p.records = drec;
    p.accum = getenv("SSA_POST_ACCUM") ? atoi(getenv("SSA_POST_ACCUM")) : 1;
    auto timed = [&]() {
      for (int i = 0; i < 3; ++i) postprocess(p, s);
      chk(hipEventRecord(e0, s), "rec");
      for (int i = 0; i < reps; ++i) postprocess(p, s);
      chk(hipEventRecord(e1, s), "rec");
      chk(hipEventSynchronize(e1), "sync");
      float ms = 0;
      chk(hipEventElapsedTime(&ms, e0, e1), "elapsed");
      return ms;
    };
    if (getenv("SSA_POST_STAGEWISE")) {  // debug builds: cumulative time of the first n launches
      float prev = 0;
      for (int n = 1; n <= 5; ++n) {
        char v[8];
        snprintf(v, sizeof v, "%d", n);
        setenv("SSA_POST_STAGES", v, 1);
        const float t = timed() * 1e3f / reps;
        printf("  %-8s stages<=%d %8.1f us/call (+%.1f)\n", names[kind], n, t, t - prev);
        prev = t;
      }
      unsetenv("SSA_POST_STAGES");
    }
    const float ms = timed();
    chk(hipMemcpy(rec.data(), drec, rec.size() * 4, hipMemcpyDeviceToHost), "rec");
    double nrec = 0, chks = 0;
    for (int b = 0; b < B; ++b) {
      const float* r = rec.data() + (size_t)b * (1 + 5 * K);
      const int n = (int)std::fabs(r[0]);
      nrec += n;
      for (int j = 0; j < 5 * n; ++j) chks += r[1 + j] * (1 + (j % 7));
    }
    printf("%-8s %8.1f us/call  records %4.0f  checksum %.6f\n", names[kind], ms * 1e3 / reps, nrec, chks);
  }
  return 0;
}
