// Exact host contour analysis. See contours.h for the semantics being matched.
#include "contours.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace ssa {
namespace {

// Direction codes, counter-clockwise on screen (y grows downwards):
// 0 right, 1 up-right, 2 up, 3 up-left, 4 left, 5 down-left, 6 down, 7 down-right.
constexpr int kDX[8] = {1, 1, 0, -1, -1, -1, 0, 1};
constexpr int kDY[8] = {0, -1, -1, -1, 0, 1, 1, 1};

struct Border {
  bool is_hole;
  int parent;                 // border number of the parent (1 = frame)
  std::vector<int> children;  // head-inserted: newest first
  int out_index = -1;
  Contour c;
};

// Padded int image: value 0 background, 1 unvisited foreground, +/-nbd marked.
struct Img {
  int W, H;  // padded dims
  std::vector<int> v;
  int& at(int x, int y) { return v[(size_t)y * W + x]; }
};

void trace(Img& img, int x0, int y0, bool is_hole, int nbd, Contour& out) {
  int s = is_hole ? 0 : 4;
  const int s_start = s;
  int x1 = 0, y1 = 0;
  do {
    s = (s - 1) & 7;
    x1 = x0 + kDX[s];
    y1 = y0 + kDY[s];
  } while (img.at(x1, y1) == 0 && s != s_start);

  if (s == s_start && img.at(x1, y1) == 0) {  // isolated pixel
    img.at(x0, y0) = -nbd;
    out.chain.push_back({x0 - 1, y0 - 1});
    out.simple.push_back({x0 - 1, y0 - 1});
    return;
  }
  int x3 = x0, y3 = y0;
  int prev_s = s ^ 4;
  for (;;) {
    const int s_end = s;
    int x4 = x3, y4 = y3;
    int k = s;
    while (k < 15) {
      ++k;
      x4 = x3 + kDX[k & 7];
      y4 = y3 + kDY[k & 7];
      if (img.at(x4, y4) != 0) break;
    }
    s = k & 7;
    if ((unsigned)(s - 1) < (unsigned)s_end) {
      img.at(x3, y3) = -nbd;               // right neighbour examined and zero
    } else if (img.at(x3, y3) == 1) {
      img.at(x3, y3) = nbd;
    }
    out.chain.push_back({x3 - 1, y3 - 1});  // back to unpadded coordinates
    if (s != prev_s) {
      out.simple.push_back({x3 - 1, y3 - 1});
      prev_s = s;
    }
    if (x4 == x0 && y4 == y0 && x3 == x1 && y3 == y1) break;
    x3 = x4;
    y3 = y4;
    s = (s + 4) & 7;
  }
}

void preorder(std::vector<Border>& b, int node, std::vector<int>& order) {
  for (int ch : b[node].children) {
    order.push_back(ch);
    preorder(b, ch, order);
  }
}

inline int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

}  // namespace

std::vector<Contour> find_contours_tree(const uint8_t* mask, int H, int W, int stride) {
  Img img{W + 2, H + 2, std::vector<int>((size_t)(W + 2) * (H + 2), 0)};
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x)
      if (mask[(size_t)y * stride + x]) img.at(x + 1, y + 1) = 1;

  // borders[0] unused, borders[1] = frame (acts as a hole border).
  std::vector<Border> borders(2);
  borders[1].is_hole = true;
  borders[1].parent = 0;
  int nbd = 1;

  for (int y = 1; y <= H; ++y) {
    int lnbd = 1;
    for (int x = 1; x <= W; ++x) {
      const int p = img.at(x, y);
      if (p == 0) {
        // hole border starts at the foreground pixel on our left
        const int prev = img.at(x - 1, y);
        if (prev >= 1) {
          ++nbd;
          Border nb;
          nb.is_hole = true;
          const Border& lb = borders[lnbd];
          nb.parent = lb.is_hole ? lb.parent : lnbd;  // hole-hole -> parent(LNBD)
          if (nb.parent == 0) nb.parent = 1;
          nb.c.is_hole = true;
          nb.c.start = {x - 2, y - 1};
          borders.push_back(std::move(nb));
          trace(img, x - 1, y, true, nbd, borders[nbd].c);
          borders[borders[nbd].parent].children.insert(
              borders[borders[nbd].parent].children.begin(), nbd);
          lnbd = nbd;  // OpenCV: lnbd.x = x - is_hole (the start pixel)
        }
        continue;
      }
      const int prev = img.at(x - 1, y);
      if (p == 1 && prev == 0) {
        ++nbd;
        Border nb;
        nb.is_hole = false;
        const Border& lb = borders[lnbd];
        nb.parent = lb.is_hole ? lnbd : lb.parent;  // outer-outer -> parent(LNBD)
        if (nb.parent == 0) nb.parent = 1;
        nb.c.is_hole = false;
        nb.c.start = {x - 1, y - 1};
        borders.push_back(std::move(nb));
        trace(img, x, y, false, nbd, borders[nbd].c);
        borders[borders[nbd].parent].children.insert(
            borders[borders[nbd].parent].children.begin(), nbd);
      }
      const int v = img.at(x, y);
      if (v != 1 && v != 0) lnbd = std::abs(v);
    }
  }

  std::vector<int> order;
  preorder(borders, 1, order);
  for (size_t i = 0; i < order.size(); ++i) borders[order[i]].out_index = (int)i;
  std::vector<Contour> out;
  out.reserve(order.size());
  for (int id : order) {
    Contour c = std::move(borders[id].c);
    const int par = borders[id].parent;
    c.parent = par <= 1 ? -1 : borders[par].out_index;
    out.push_back(std::move(c));
  }
  return out;
}

double contour_area(const std::vector<Pt>& pts) {
  const size_t n = pts.size();
  if (n == 0) return 0.0;
  double a00 = 0;
  Pt prev = pts[n - 1];
  for (size_t i = 0; i < n; ++i) {
    const Pt p = pts[i];
    a00 += (double)prev.x * p.y - (double)prev.y * p.x;
    prev = p;
  }
  return std::fabs(a00 * 0.5);
}

Moments contour_moments(const std::vector<Pt>& pts) {
  Moments m;
  const size_t n = pts.size();
  if (n == 0) return m;
  double a00 = 0, a10 = 0, a01 = 0;
  double xi_1 = pts[n - 1].x, yi_1 = pts[n - 1].y;
  for (size_t i = 0; i < n; ++i) {
    const double xi = pts[i].x, yi = pts[i].y;
    const double dxy = xi_1 * yi - xi * yi_1;
    a00 += dxy;
    a10 += dxy * (xi_1 + xi);
    a01 += dxy * (yi_1 + yi);
    xi_1 = xi;
    yi_1 = yi;
  }
  m.a00 = a00;
  m.a10 = a10;
  m.a01 = a01;
  if (std::fabs(a00) > 1.1920928955078125e-07) {  // FLT_EPSILON
    const double db1_2 = a00 > 0 ? 0.5 : -0.5;
    const double db1_6 = a00 > 0 ? 0.16666666666666666666666666666667
                                 : -0.16666666666666666666666666666667;
    m.m00 = a00 * db1_2;
    m.m10 = a10 * db1_6;
    m.m01 = a01 * db1_6;
  }
  return m;
}

void fill_contour(const std::vector<Pt>& pts, int H, int W, uint8_t* out) {
  const size_t n = pts.size();
  if (n == 0) return;
  // Boundary: consecutive simplified vertices are joined by straight 8-direction
  // runs, so stepping one unit at a time reproduces the rasterised line.
  for (size_t i = 0; i < n; ++i) {
    Pt a = pts[i], b = pts[(i + 1) % n];
    const int sx = (b.x > a.x) - (b.x < a.x), sy = (b.y > a.y) - (b.y < a.y);
    for (;;) {
      if (a.x >= 0 && a.x < W && a.y >= 0 && a.y < H) out[(size_t)a.y * W + a.x] = 255;
      if (a.x == b.x && a.y == b.y) break;
      // a straight run in one of the 8 directions
      if (a.x != b.x) a.x += sx;
      if (a.y != b.y) a.y += sy;
    }
  }
  // Interior: even-odd scanlines at y + epsilon (pixel centres on integer lattice).
  int ymin = pts[0].y, ymax = pts[0].y;
  for (const Pt& p : pts) { ymin = std::min(ymin, p.y); ymax = std::max(ymax, p.y); }
  std::vector<double> xs;
  for (int y = std::max(ymin, 0); y <= std::min(ymax, H - 1); ++y) {
    xs.clear();
    for (size_t i = 0; i < n; ++i) {
      const Pt a = pts[i], b = pts[(i + 1) % n];
      if (a.y == b.y) continue;
      const int lo = std::min(a.y, b.y), hi = std::max(a.y, b.y);
      if (y < lo || y >= hi) continue;
      // crossing of the line y + 0.5 * (tiny) -> evaluate at y exactly, lines are
      // straight runs so x is linear in y
      const double t = (double)(y - a.y) / (double)(b.y - a.y);
      const double tx = a.x + t * (b.x - a.x);
      // nudge by the edge slope for the y+eps evaluation
      const double slope = (double)(b.x - a.x) / (double)(b.y - a.y);
      xs.push_back(tx + slope * 1e-6);
    }
    std::sort(xs.begin(), xs.end());
    for (size_t k = 0; k + 1 < xs.size(); k += 2) {
      const int xa = std::max(0, (int)std::ceil(xs[k]));
      const int xb = std::min(W - 1, (int)std::floor(xs[k + 1]));
      for (int x = xa; x <= xb; ++x) out[(size_t)y * W + x] = 255;
    }
  }
}

void palette_mask(const uint8_t* labels, int h, int w, int ls, const int32_t* palette,
                  int thr, uint8_t* out) {
  for (int y = 0; y < h; ++y) {
    for (int x = 0; x < w; ++x) {
      int sum[3] = {0, 0, 0};
      for (int dy = -1; dy <= 1; ++dy) {
        const int yy = reflect101(y + dy, h);
        for (int dx = -1; dx <= 1; ++dx) {
          const int xx = reflect101(x + dx, w);
          const int l = labels[(size_t)yy * ls + xx];
          sum[0] += palette[l * 3 + 0];
          sum[1] += palette[l * 3 + 1];
          sum[2] += palette[l * 3 + 2];
        }
      }
      // round(sum / 9); sum/9 never lands on .5 so rounding mode is moot
      const int c0 = (sum[0] * 2 + 9) / 18, c1 = (sum[1] * 2 + 9) / 18, c2 = (sum[2] * 2 + 9) / 18;
      // BGR2GRAY on RGB data: channel 0 gets the blue weight
      const int g = (c0 * 1868 + c1 * 9617 + c2 * 4899 + (1 << 13)) >> 14;
      out[(size_t)y * w + x] = g > thr ? 255 : 0;
    }
  }
}

std::vector<Segment> segments_exact(const uint8_t* labels, int h, int w, int ls,
                                    const int32_t* palette, double min_area, int num_bins) {
  std::vector<Segment> segs;
  if (h <= 0 || w <= 0) return segs;
  std::vector<uint8_t> mask((size_t)h * w);
  palette_mask(labels, h, w, ls, palette, 127, mask.data());
  std::vector<Contour> cs = find_contours_tree(mask.data(), h, w, w);
  std::vector<uint8_t> fill((size_t)h * w);
  std::vector<long long> hist(256);
  for (size_t i = 0; i < cs.size(); ++i) {
    const double area = contour_area(cs[i].simple);
    if (area < min_area) continue;
    std::fill(fill.begin(), fill.end(), 0);
    fill_contour(cs[i].simple, h, w, fill.data());
    std::fill(hist.begin(), hist.end(), 0);
    long long n = 0;
    int maxl = 0;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x)
        if (fill[(size_t)y * w + x]) {
          const int l = labels[(size_t)y * ls + x];
          ++hist[l];
          ++n;
          maxl = std::max(maxl, l);
        }
    int best = 0;
    for (int l = 1; l <= maxl; ++l)
      if (hist[l] > hist[best]) best = l;
    const Moments m = contour_moments(cs[i].simple);
    if (m.m00 == 0.0) continue;
    Segment s;
    s.label = best;
    s.score = (double)hist[best] / (double)n;
    s.area = area;
    s.cx = (int)(m.m10 / m.m00);
    s.cy = (int)(m.m01 / m.m00);
    s.contour = (int)i;
    s.is_hole = cs[i].is_hole;
    segs.push_back(s);
  }
  (void)num_bins;
  return segs;
}

}  // namespace ssa
