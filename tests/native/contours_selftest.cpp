// Sanitizer self-test of the host contour oracle: built with
// -fsanitize=address,undefined by tests/test_native_sanitizers.py and run over
// random label maps. Checks invariants that hold for any correct findContours:
//   * every contour's parent index precedes it (pre-order) and holes alternate
//     with outer borders along the parent chain;
//   * every chain pixel lies inside the image and on the foreground (outer
//     borders) / background-adjacent side as the mask says;
//   * contour_area(simple) == contour_area(chain) (CHAIN_APPROX_SIMPLE only drops
//     collinear points);
//   * segments_exact scores are in (0, 1] and centroids inside the crop.
// Any out-of-bounds access or UB in the tracer aborts under the sanitizers.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "contours.h"

using namespace ssa;

static int fail(const char* what, int it) {
  std::fprintf(stderr, "FAIL %s (iteration %d)\n", what, it);
  return 1;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
  std::mt19937 rng(1234);
  std::vector<int32_t> pal(256 * 3, 0);
  pal[7 * 3 + 0] = 128; pal[7 * 3 + 1] = 128; pal[7 * 3 + 2] = 128;    // car
  pal[15 * 3 + 0] = 192; pal[15 * 3 + 1] = 128; pal[15 * 3 + 2] = 128; // person
  for (int it = 0; it < iters; ++it) {
    const int h = 1 + rng() % 70, w = 1 + rng() % 70;
    std::vector<uint8_t> lab(h * w, 0);
    const int blobs = rng() % 6;
    for (int b = 0; b < blobs; ++b) {
      const int cy = rng() % h, cx = rng() % w, ry = 1 + rng() % (h / 2 + 1), rx = 1 + rng() % (w / 2 + 1);
      const int cls = (rng() % 2) ? 15 : 7;
      for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
          const double e = double(y - cy) * (y - cy) / (ry * ry) + double(x - cx) * (x - cx) / (rx * rx);
          if (e < 1.0) lab[y * w + x] = (e < 0.3 && (b & 1)) ? 0 : cls;
        }
    }
    const int noise = rng() % 40;
    for (int n = 0; n < noise; ++n) lab[rng() % (h * w)] = (rng() % 2) ? 15 : 0;
    std::vector<uint8_t> mask(h * w);
    palette_mask(lab.data(), h, w, w, pal.data(), 127, mask.data());
    const auto cs = find_contours_tree(mask.data(), h, w, w);
    for (size_t i = 0; i < cs.size(); ++i) {
      const Contour& c = cs[i];
      if (c.parent >= (int)i) return fail("parent after child", it);
      if (c.parent >= 0 && cs[c.parent].is_hole == c.is_hole) return fail("hole nesting", it);
      if (c.chain.empty() || c.simple.empty()) return fail("empty contour", it);
      for (const Pt& p : c.chain) {
        if (p.x < 0 || p.y < 0 || p.x >= w || p.y >= h) return fail("chain out of image", it);
        if (!mask[p.y * w + p.x]) return fail("chain pixel not foreground", it);
      }
      if (std::fabs(contour_area(c.simple) - contour_area(c.chain)) > 1e-9)
        return fail("simple/chain area mismatch", it);
    }
    const auto segs = segments_exact(lab.data(), h, w, w, pal.data(), 0.0, 32);
    for (const Segment& s : segs) {
      if (!(s.score > 0.0 && s.score <= 1.0)) return fail("score range", it);
      if (s.cx < 0 || s.cy < 0 || s.cx >= w || s.cy >= h) return fail("centroid outside", it);
    }
  }
  std::printf("ok %d maps\n", iters);
  return 0;
}
