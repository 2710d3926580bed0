// Host-side exact contour analysis (test oracle + --contour_mode=exact).
//
// Re-implements, from the published algorithm, the semantics the reference gets
// from OpenCV 3.x (sem_seg_server.py:77-133):
//   * Suzuki & Abe (1985) border following on an 8-connected foreground /
//     4-connected background, over the image padded with one pixel of zeros
//     (findContours(RETR_TREE, CHAIN_APPROX_SIMPLE));
//   * contour order = pre-order walk of the border tree in which every newly
//     found border is inserted at the head of its parent's child list;
//   * contourArea (shoelace, |a00|/2) and contour moments (Green's theorem,
//     double accumulation, m00/m10/m01);
//   * drawContours(..., thickness=FILLED): chain pixels plus the even-odd
//     scanline interior of the polygon.
// All of this is [EXT] behaviour: OpenCV is not installable here, so parity is
// by construction and by the tests in tests/test_postprocess_parity.py.
#pragma once
#include <cstdint>
#include <vector>

namespace ssa {

struct Pt { int x, y; };

struct Contour {
  std::vector<Pt> chain;    // every border pixel visited (CHAIN_APPROX_NONE)
  std::vector<Pt> simple;   // direction-change vertices (CHAIN_APPROX_SIMPLE)
  bool is_hole = false;
  int parent = -1;          // index into the output order, -1 = top level
  Pt start{0, 0};           // first border pixel (raster discovery point)
};

// Contours of a binary image (nonzero = foreground) in OpenCV output order.
std::vector<Contour> find_contours_tree(const uint8_t* mask, int H, int W, int stride);

struct Moments { double m00 = 0, m10 = 0, m01 = 0; double a00 = 0, a10 = 0, a01 = 0; };

double contour_area(const std::vector<Pt>& pts);
Moments contour_moments(const std::vector<Pt>& pts);
// Rasterised FILLED drawing of one contour into out (H x W, set to 255).
void fill_contour(const std::vector<Pt>& pts, int H, int W, uint8_t* out);

// OpenCV-exact mask stage: palette colour -> 3x3 box blur (BORDER_REFLECT_101,
// rounded) -> fixed-point BGR2GRAY applied to RGB data -> threshold > thr.
// labels: h x w (row stride ls); palette: 256 x 3 RGB; out: h x w 0/255.
void palette_mask(const uint8_t* labels, int h, int w, int ls, const int32_t* palette,
                  int thr, uint8_t* out);

struct Segment {
  int label;        // majority class id
  double score;     // majority fraction
  double area;      // contour area in pixels^2
  int cx, cy;       // truncated polygon centroid
  int contour;      // index in contour order
  bool is_hole;
};

// Full reference post-processing of one cropped label map (sem_seg_server.py:
// 170-181 + process_segment_contours :92-133), in contour order.
std::vector<Segment> segments_exact(const uint8_t* labels, int h, int w, int ls,
                                    const int32_t* palette, double min_area, int num_bins);

}  // namespace ssa
