// Device contour statistics (K7-K10 of SURVEY.md §2.5) for gfx950.
//
// Computes, for every frame of a batch, exactly what the reference gets from
// label_to_color_image + cv2.blur/cvtColor/threshold + findContours(RETR_TREE) +
// contourArea/drawContours/bincount/moments (sem_seg_server.py:77-133,164-192),
// without tracing a single border. The math (and its proof obligations) is
// written out in semantic_segmentation_server_amd/postprocess/components.py;
// tests check these kernels against it and against the exact host tracer.
//
// Pipeline (fixed launch sequence, no host round trip, hipGraph-capturable):
//   k_ccl_local  per 32x8 tile: palette -> 3x3 box blur (REFLECT_101, rounded) ->
//                BGR2GRAY on RGB (fixed point) -> > thr, then union-find in LDS:
//                foreground 8-connected, background 4-connected
//   k_ccl_boundary  global union-find (atomicMin, Playne-Hawick style) only
//                across tile edges; image-border background joins the virtual
//                "outside" node 0
//   k_compress   label = root with path halving (root = raster index of the
//                component's first pixel + 1, 0 = outside)
//   k_roots      per component: zero accumulators, parent in the border tree
//   k_quads      per 2x2 quad: polygon pieces (full square / triangle) as exact
//                integer moments a00 = 2A, a10 = 6*int x, a01 = 6*int y
//   k_tree       subtree sums: every component adds its own pieces to all its
//                ancestors
//   k_select     contours whose polygon area >= min_area get a record slot
//   k_hist       class histogram of each selected contour's fill (component +
//                everything it encloses; holes also get the parent's ring pixels)
//   k_finalize   majority label, score, centroid (OpenCV's double arithmetic),
//                normalisation, records in findContours pre-order
#include "common.h"
#include "kernels.h"

#include <cstdlib>

namespace ssa {
namespace {

struct FrameWS {
  int32_t* L;          // [N + 1] union-find labels (index 0 = outside)
  uint8_t* mask;       // [N] 1 = foreground
  int32_t* parent;     // [N] per root index: parent node id (0 = frame/outside)
  int32_t* slot;       // [N] per root index: record slot or -1
  int32_t* a00;        // [N] own 2*area
  int32_t* t00;        // [N] subtree 2*area
  long long* a10;      // [N]
  long long* a01;      // [N]
  long long* t10;      // [N]
  long long* t01;      // [N]
  int32_t* hist;       // [K][bins]
  int32_t* nslot;      // [1] (+ overflow flag at [1])
  int32_t* slot_node;  // [K]
};

// Workspace layout: per frame, fixed stride; counters/hists first (memset region).
struct Layout {
  size_t N, K, bins;
  size_t small_bytes;  // nslot(16) + hist + slot_node, per frame (zeroed every call)
  size_t big_bytes;    // per frame
  size_t total(int B) const { return (small_bytes + big_bytes) * (size_t)B; }
};

__host__ __device__ inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

Layout layout(int H, int W, int K, int bins) {
  Layout l;
  l.N = (size_t)H * W;
  l.K = K;
  l.bins = bins;
  l.small_bytes = al(16 + (size_t)K * bins * 4 + (size_t)K * 4);
  l.big_bytes = al((l.N + 1) * 4) + al(l.N) + 4 * al(l.N * 4) + 4 * al(l.N * 8);
  return l;
}

__host__ __device__ inline FrameWS frame_ws(char* ws, const Layout& l, int B, int b) {
  FrameWS f;
  char* s = ws + (size_t)b * l.small_bytes;
  f.nslot = reinterpret_cast<int32_t*>(s);
  f.hist = reinterpret_cast<int32_t*>(s + 16);
  f.slot_node = reinterpret_cast<int32_t*>(s + 16 + l.K * l.bins * 4);
  char* p = ws + (size_t)B * l.small_bytes + (size_t)b * l.big_bytes;
  f.L = reinterpret_cast<int32_t*>(p); p += al((l.N + 1) * 4);
  f.mask = reinterpret_cast<uint8_t*>(p); p += al(l.N);
  f.parent = reinterpret_cast<int32_t*>(p); p += al(l.N * 4);
  f.slot = reinterpret_cast<int32_t*>(p); p += al(l.N * 4);
  f.a00 = reinterpret_cast<int32_t*>(p); p += al(l.N * 4);
  f.t00 = reinterpret_cast<int32_t*>(p); p += al(l.N * 4);
  f.a10 = reinterpret_cast<long long*>(p); p += al(l.N * 8);
  f.a01 = reinterpret_cast<long long*>(p); p += al(l.N * 8);
  f.t10 = reinterpret_cast<long long*>(p); p += al(l.N * 8);
  f.t01 = reinterpret_cast<long long*>(p); p += al(l.N * 8);
  return f;
}

struct KArgs {
  const uint8_t* labels;  // [B, H, W]
  int B, H, W, ch, cw, thr, K, bins;
  double min_area;
  char* ws;
  Layout lay;
  float* records;
};

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i;
}

__device__ __forceinline__ int ld_relaxed(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ int find_root(int32_t* L, int x) {
  int y = ld_relaxed(L + x);
  while (y != x) {
    x = y;
    y = ld_relaxed(L + x);
  }
  return x;
}

__device__ __forceinline__ int find_halving(int32_t* L, int x) {
  int y = ld_relaxed(L + x);
  while (y != x) {
    const int z = ld_relaxed(L + y);
    if (z != y) __hip_atomic_store(L + x, z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x = y;
    y = z;
  }
  return x;
}

__device__ void unite(int32_t* L, int a, int b) {
  for (int guard = 0; guard < (1 << 24); ++guard) {
    a = find_halving(L, a);
    b = find_halving(L, b);
    if (a == b) return;
    if (a < b) {
      const int old = atomicMin(L + b, a);
      if (old == b) return;
      b = old;
    } else {
      const int old = atomicMin(L + a, b);
      if (old == a) return;
      a = old;
    }
  }
}

// ---------------------------------------------------------------- mask + local CCL
// One 256-thread block = one TW x TH pixel tile. Each thread computes its pixel's
// mask bit (palette -> 3x3 blur -> gray -> threshold) and the tile's connected
// components are resolved with union-find on LDS labels; the global label of a
// pixel is then the raster index (+1) of its tile-local root, which is also the
// tile-local minimum, so the global min-root invariant is preserved.
constexpr int TW = 32, TH = 8;

__device__ __forceinline__ int lds_ld(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ int lfind(int* l, int x) {
  int y = lds_ld(l + x);
  while (y != x) {
    x = y;
    y = lds_ld(l + x);
  }
  return x;
}

__device__ void lunite(int* l, int a, int b) {
  for (;;) {
    a = lfind(l, a);
    b = lfind(l, b);
    if (a == b) return;
    if (a < b) {
      const int old = atomicMin(l + b, a);
      if (old == b) return;
      b = old;
    } else {
      const int old = atomicMin(l + a, b);
      if (old == a) return;
      a = old;
    }
  }
}

__global__ __launch_bounds__(256) void k_ccl_local(KArgs a, const int32_t* __restrict__ pal) {
  __shared__ int spal[256 * 3];
  __shared__ int lbl[TW * TH];
  __shared__ uint8_t msk[TW * TH];
  for (int i = threadIdx.x; i < 256 * 3; i += blockDim.x) spal[i] = pal[i];
  const int b = blockIdx.z;
  const int tx = threadIdx.x % TW, ty = threadIdx.x / TW;
  const int x = blockIdx.x * TW + tx, y = blockIdx.y * TH + ty;
  const bool in = x < a.cw && y < a.ch;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) f.L[0] = 0;
  __syncthreads();
  uint8_t m = 0;
  if (in) {
    const uint8_t* lab = a.labels + (size_t)b * a.H * a.W;
    int s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int yy = reflect101(y + dy, a.ch);
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int xx = reflect101(x + dx, a.cw);
        const int l = lab[yy * a.W + xx];
        s0 += spal[l * 3 + 0];
        s1 += spal[l * 3 + 1];
        s2 += spal[l * 3 + 2];
      }
    }
    const int c0 = (s0 * 2 + 9) / 18, c1 = (s1 * 2 + 9) / 18, c2 = (s2 * 2 + 9) / 18;
    const int g = (c0 * 1868 + c1 * 9617 + c2 * 4899 + (1 << 13)) >> 14;
    m = g > a.thr ? 1 : 0;
    f.mask[y * a.cw + x] = m;
  }
  const int me = threadIdx.x;
  msk[me] = in ? m : 2;  // 2 = outside the crop (never joins anything)
  lbl[me] = me;
  __syncthreads();
  if (in) {
    if (m) {
      if (tx > 0 && msk[me - 1] == 1) lunite(lbl, me, me - 1);
      if (ty > 0) {
        const int up = me - TW;
        if (msk[up] == 1) lunite(lbl, me, up);
        if (tx > 0 && msk[up - 1] == 1) lunite(lbl, me, up - 1);
        if (tx + 1 < TW && msk[up + 1] == 1) lunite(lbl, me, up + 1);
      }
    } else {
      if (tx > 0 && msk[me - 1] == 0) lunite(lbl, me, me - 1);
      if (ty > 0 && msk[me - TW] == 0) lunite(lbl, me, me - TW);
    }
  }
  __syncthreads();
  if (in) {
    const int r = lfind(lbl, me);
    const int rx = blockIdx.x * TW + r % TW, ry = blockIdx.y * TH + r / TW;
    f.L[y * a.cw + x + 1] = ry * a.cw + rx + 1;
  }
}

// Cross-tile merges (and image-border background -> outside node 0). Only
// pixels on a tile's left column / top row or on the image border do work.
__global__ __launch_bounds__(256) void k_ccl_boundary(KArgs a) {
  const int b = blockIdx.y;
  const int N = a.ch * a.cw;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= N) return;
  const int y = p / a.cw, x = p - y * a.cw;
  const bool left = x > 0 && (x % TW) == 0;
  const bool top = y > 0 && (y % TH) == 0;
  const bool edge = x == 0 || y == 0 || x == a.cw - 1 || y == a.ch - 1;
  const bool rtile = (x % TW) == TW - 1 && x + 1 < a.cw && y > 0;  // up-right neighbour in next tile
  if (!left && !top && !edge && !rtile) return;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  const uint8_t m = f.mask[p];
  const int me = p + 1;
  // Skip unions already implied by the previous pixel along the same tile edge:
  // if it has the same class, the same tile-local root and its partner across the
  // edge has the same local root as ours, it issued the identical union. (Local
  // roots are still in L: tile-local writes are the only writes before this pass
  // apart from root links, which keep equal roots equal.)
  auto lroot = [&](int q) { return f.L[q + 1]; };
  if (m) {
    if (left && f.mask[p - 1]) unite(f.L, me, me - 1);
    if (y > 0) {
      const int up = p - a.cw;
      if (top) {
        const bool dup = x > 0 && (x % TW) != 0 && f.mask[p - 1] && lroot(p - 1) == lroot(p);
        if (f.mask[up] && !(dup && f.mask[up - 1] && lroot(up - 1) == lroot(up)))
          unite(f.L, me, up + 1);
        if (x > 0 && f.mask[up - 1]) unite(f.L, me, up);
        if (x + 1 < a.cw && f.mask[up + 1]) unite(f.L, me, up + 2);
      } else {
        // same tile row: diagonals that cross a vertical tile edge
        if (left && f.mask[up - 1]) unite(f.L, me, up);
        if (rtile && f.mask[up + 1]) unite(f.L, me, up + 2);
      }
    }
  } else {
    if (left && !f.mask[p - 1]) {
      const bool dup = y > 0 && (y % TH) != 0 && !f.mask[p - a.cw] && !f.mask[p - a.cw - 1] &&
                       lroot(p - a.cw) == lroot(p) && lroot(p - a.cw - 1) == lroot(p - 1);
      if (!dup) unite(f.L, me, me - 1);
    }
    if (top && !f.mask[p - a.cw]) {
      const bool dup = x > 0 && (x % TW) != 0 && !f.mask[p - 1] && !f.mask[p - a.cw - 1] &&
                       lroot(p - 1) == lroot(p) && lroot(p - a.cw - 1) == lroot(p - a.cw);
      if (!dup) unite(f.L, me, me - a.cw);
    }
    if (edge) {
      // one union per run of border pixels sharing a tile-local root
      const int prev = (y == 0 || y == a.ch - 1) ? (x > 0 && (x % TW) != 0 ? p - 1 : -1)
                                                 : ((y % TH) != 0 ? p - a.cw : -1);
      if (prev < 0 || f.mask[prev] || lroot(prev) != lroot(p)) unite(f.L, me, 0);
    }
  }
}

__global__ __launch_bounds__(256) void k_compress(KArgs a) {
  const int b = blockIdx.y;
  const int N = a.ch * a.cw;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= N) return;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  // Read-only traversal: a path-halving store here could overwrite another
  // thread's final root store with a stale grandparent (observed: 1 pixel in ~1M
  // left pointing at a non-root). Every concurrent store below writes a root, so
  // plain traversal always terminates at the true root.
  const int r = find_root(f.L, p + 1);
  __hip_atomic_store(f.L + p + 1, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- roots
__global__ __launch_bounds__(256) void k_roots(KArgs a) {
  const int b = blockIdx.y;
  const int N = a.ch * a.cw;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= N) return;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  if (f.L[p + 1] != p + 1) return;  // not a root (or outside)
  const int x = p % a.cw;
  // parent = component of the left neighbour of the first pixel (0 at the border)
  f.parent[p] = x > 0 ? f.L[p] : 0;
  f.slot[p] = -1;
  f.a00[p] = 0;
  f.t00[p] = 0;
  f.a10[p] = 0;
  f.a01[p] = 0;
  f.t10[p] = 0;
  f.t01[p] = 0;
}

// Wave-aggregated atomic adds: the common case is a whole wave contributing to
// the same node (interior of a large blob).
__device__ __forceinline__ void agg_add(FrameWS& f, int node, int d00, long long d10,
                                        long long d01) {
  const bool active = node > 0;
  const unsigned long long act = __ballot(active);
  if (act == 0) return;
  const int leader = __ffsll((long long)act) - 1;
  const int lnode = __shfl(node, leader, 64);
  const bool same = __all(!active || node == lnode);
  if (same) {
    int s00 = active ? d00 : 0;
    long long s10 = active ? d10 : 0, s01 = active ? d01 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s00 += __shfl_xor(s00, o, 64);
      s10 += __shfl_xor(s10, o, 64);
      s01 += __shfl_xor(s01, o, 64);
    }
    if ((int)(threadIdx.x & 63) == leader) {
      atomicAdd(f.a00 + lnode - 1, s00);
      atomicAdd(reinterpret_cast<unsigned long long*>(f.a10 + lnode - 1), (unsigned long long)s10);
      atomicAdd(reinterpret_cast<unsigned long long*>(f.a01 + lnode - 1), (unsigned long long)s01);
    }
  } else if (active) {
    atomicAdd(f.a00 + node - 1, d00);
    atomicAdd(reinterpret_cast<unsigned long long*>(f.a10 + node - 1), (unsigned long long)d10);
    atomicAdd(reinterpret_cast<unsigned long long*>(f.a01 + node - 1), (unsigned long long)d01);
  }
}

// ---------------------------------------------------------------- quads
// Corner order TL, TR, BL, BR. Triangle of corner k = k + its two quad
// neighbours; sums of its 3 vertices' coordinates = 3x + TX[k], 3y + TY[k].
__global__ __launch_bounds__(256) void k_quads(KArgs a) {
  const int b = blockIdx.y;
  const int QW = a.cw - 1, QH = a.ch - 1;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  int fnode = 0, f00 = 0;
  long long f10 = 0, f01 = 0;
  int bn[2] = {0, 0}, b00[2] = {0, 0};
  long long b10[2] = {0, 0}, b01[2] = {0, 0};
  if (QW > 0 && QH > 0 && q < QW * QH) {
    const int y = q / QW, x = q - y * QW;
    const int p0 = y * a.cw + x;
    const int idx[4] = {p0, p0 + 1, p0 + a.cw, p0 + a.cw + 1};
    const int TX[4] = {1, 2, 1, 2}, TY[4] = {1, 1, 2, 2};
    int node[4];
    bool fg[4];
    int nf = 0, missing = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      fg[k] = f.mask[idx[k]] != 0;
      node[k] = f.L[idx[k] + 1];
      if (fg[k]) { ++nf; fnode = node[k]; } else { missing = k; }
    }
    const long long X = x, Y = y;
    if (nf == 4) {
      f00 = 2; f10 = 6 * X + 3; f01 = 6 * Y + 3;
    } else if (nf == 3) {
      const int o = 3 - missing;  // triangle of the opposite corner
      f00 = 1; f10 = 3 * X + TX[o]; f01 = 3 * Y + TY[o];
    } else {
      fnode = 0;
    }
    int nb = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (fg[k] || node[k] == 0) continue;
      bool first = true;
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!fg[j] && node[j] == node[k]) {
          ++cnt;
          if (j < k) first = false;
        }
      }
      if (!first) continue;
      if (nb < 2) {
        bn[nb] = node[k];
        if (cnt >= 2) { b00[nb] = 2; b10[nb] = 6 * X + 3; b01[nb] = 6 * Y + 3; }
        else { b00[nb] = 1; b10[nb] = 3 * X + TX[k]; b01[nb] = 3 * Y + TY[k]; }
        ++nb;
      }
    }
  }
  agg_add(f, fnode, f00, f10, f01);
  agg_add(f, bn[0], b00[0], b10[0], b01[0]);
  agg_add(f, bn[1], b00[1], b10[1], b01[1]);
}

// ---------------------------------------------------------------- tree sums
__global__ __launch_bounds__(256) void k_tree(KArgs a) {
  const int b = blockIdx.y;
  const int N = a.ch * a.cw;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= N) return;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  if (f.L[p + 1] != p + 1) return;
  const int o00 = f.a00[p];
  const long long o10 = f.a10[p], o01 = f.a01[p];
  if (o00 == 0 && o10 == 0 && o01 == 0) return;
  int n = p + 1;
  for (int depth = 0; n != 0 && depth < 65536; ++depth) {
    atomicAdd(f.t00 + n - 1, o00);
    atomicAdd(reinterpret_cast<unsigned long long*>(f.t10 + n - 1), (unsigned long long)o10);
    atomicAdd(reinterpret_cast<unsigned long long*>(f.t01 + n - 1), (unsigned long long)o01);
    n = f.parent[n - 1];
  }
}

// ---------------------------------------------------------------- select
__global__ __launch_bounds__(256) void k_select(KArgs a) {
  const int b = blockIdx.y;
  const int N = a.ch * a.cw;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= N) return;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  if (f.L[p + 1] != p + 1) return;
  const double area = (double)f.t00[p] * 0.5;
  if (!(area >= a.min_area) || f.t00[p] == 0) return;
  const int s = atomicAdd(f.nslot, 1);
  if (s < a.K) {
    f.slot[p] = s;
    f.slot_node[s] = p + 1;
  } else {
    f.nslot[1] = 1;  // overflow: contour dropped
  }
}

// ---------------------------------------------------------------- histograms
__device__ __forceinline__ void hist_add(int32_t* hist, int bins, int slot, int label) {
  // aggregate identical (slot, label) pairs across the wave
  const int key = slot >= 0 ? slot * bins + label : -1;
  const unsigned long long act = __ballot(key >= 0);
  if (act == 0) return;
  const int leader = __ffsll((long long)act) - 1;
  const int lkey = __shfl(key, leader, 64);
  if (__all(key < 0 || key == lkey)) {
    if ((int)(threadIdx.x & 63) == leader) atomicAdd(hist + lkey, __popcll(act));
  } else if (key >= 0) {
    atomicAdd(hist + key, 1);
  }
}

__global__ __launch_bounds__(256) void k_hist(KArgs a) {
  const int b = blockIdx.y;
  const int N = a.ch * a.cw;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  if (*f.nslot == 0) return;  // block-uniform early exit: no contour selected
  int label = 0, n = 0, y = 0, x = 0;
  bool fgp = false;
  if (p < N) {
    y = p / a.cw;
    x = p - y * a.cw;
    label = a.labels[(size_t)b * a.H * a.W + y * a.W + x];
    if (label >= a.bins) label = a.bins - 1;
    n = f.L[p + 1];
    fgp = f.mask[p] != 0;
  }
  // ancestors (inclusive): the fill of every enclosing contour contains p
  int depth = 0;
  while (true) {
    const int s = (n != 0) ? f.slot[n - 1] : -1;
    const bool more = __any(n != 0);
    if (!more) break;
    hist_add(f.hist, a.bins, s, label);
    if (n != 0) n = f.parent[n - 1];
    if (++depth > 65536) break;
  }
  // ring: a foreground pixel 4-adjacent to a selected hole of its own component
  int hs[4] = {-1, -1, -1, -1};
  if (p < N && fgp) {
    const int me = f.L[p + 1];
    const int nb[4] = {x > 0 ? p - 1 : -1, x + 1 < a.cw ? p + 1 : -1, y > 0 ? p - a.cw : -1,
                       y + 1 < a.ch ? p + a.cw : -1};
    int seen[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (nb[k] < 0 || f.mask[nb[k]]) continue;
      const int h = f.L[nb[k] + 1];
      if (h == 0 || f.parent[h - 1] != me) continue;
      bool dup = false;
      for (int j = 0; j < k; ++j) dup |= (seen[j] == h);
      seen[k] = h;
      if (!dup) hs[k] = f.slot[h - 1];
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) hist_add(f.hist, a.bins, hs[k], label);
}

// ---------------------------------------------------------------- finalize
constexpr int kMaxDepth = 32;

__global__ __launch_bounds__(64) void k_finalize(KArgs a) {
  const int b = blockIdx.x;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  float* rec = a.records + (size_t)b * (1 + 5 * a.K);
  __shared__ int s_node[256];
  __shared__ int s_path[256][kMaxDepth];
  __shared__ int s_len[256];
  __shared__ int s_order[256];
  __shared__ int s_emit[256];
  __shared__ float s_val[256][5];
  const int ns = min(*f.nslot, min(a.K, 256));
  const int t = threadIdx.x;
  for (int i = t; i < ns; i += 64) {
    const int node = f.slot_node[i];
    s_node[i] = node;
    // ancestor chain (top first) of discovery keys
    int chain[kMaxDepth];
    int len = 0;
    for (int n = node; n != 0 && len < kMaxDepth; n = f.parent[n - 1]) {
      const int r = n - 1;
      const bool isfg = f.mask[r] != 0;
      chain[len++] = isfg ? r : r - 1;
    }
    for (int k = 0; k < len; ++k) s_path[i][k] = chain[len - 1 - k];
    s_len[i] = len;
    // statistics
    const int r = node - 1;
    const int* h = f.hist + (size_t)i * a.bins;
    int best = 0, tot = 0;
    for (int c = 0; c < a.bins; ++c) {
      tot += h[c];
      if (h[c] > h[best]) best = c;
    }
    const double a00 = (double)f.t00[r];
    const double m00 = a00 * 0.5;
    const double m10 = (double)f.t10[r] * 0.16666666666666666666666666666667;
    const double m01 = (double)f.t01[r] * 0.16666666666666666666666666666667;
    const bool ok = m00 != 0.0 && tot > 0;
    s_emit[i] = ok;
    if (ok) {
      const int cx = (int)(m10 / m00);
      const int cy = (int)(m01 / m00);
      const double area = m00;  // |a00| / 2
      s_val[i][0] = (float)best;
      s_val[i][1] = (float)((double)h[best] / (double)tot);
      s_val[i][2] = (float)fmin(1.0, area / ((double)a.W * (double)a.H));
      s_val[i][3] = (float)fmin(1.0, (double)cx / (double)a.W);
      s_val[i][4] = (float)fmin(1.0, (double)cy / (double)a.H);
    }
  }
  __syncthreads();
  // rank in pre-order: ancestor first; siblings by descending discovery key
  for (int i = t; i < ns; i += 64) {
    int rank = 0;
    for (int j = 0; j < ns; ++j) {
      if (j == i) continue;
      // does j come before i?
      const int li = s_len[i], lj = s_len[j];
      int k = 0;
      while (k < li && k < lj && s_path[i][k] == s_path[j][k]) ++k;
      bool before;
      if (k == lj) before = true;        // j is an ancestor of i
      else if (k == li) before = false;  // i is an ancestor of j
      else before = s_path[j][k] > s_path[i][k];
      rank += before;
    }
    s_order[rank] = i;
  }
  __syncthreads();
  if (t == 0) {
    int n = 0;
    for (int r = 0; r < ns; ++r) {
      const int i = s_order[r];
      if (!s_emit[i]) continue;
      for (int c = 0; c < 5; ++c) rec[1 + 5 * n + c] = s_val[i][c];
      ++n;
    }
    rec[0] = (float)n;
  }
}

__global__ __launch_bounds__(256) void k_zero(uint4* __restrict__ p, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(0, 0, 0, 0);
}

}  // namespace

size_t post_workspace_bytes(int B, int H, int W, int K, int num_bins) {
  return layout(H, W, K, num_bins).total(B);
}

void postprocess(const PostParams& p, hipStream_t s) {
  if (p.K > 256) throw std::invalid_argument("postprocess: K > 256");
  if (p.crop_h > p.H || p.crop_w > p.W || p.crop_h <= 0 || p.crop_w <= 0)
    throw std::invalid_argument("postprocess: bad crop");
  KArgs a;
  a.labels = p.labels;
  a.B = p.B; a.H = p.H; a.W = p.W; a.ch = p.crop_h; a.cw = p.crop_w;
  a.thr = p.thr; a.K = p.K; a.bins = p.num_bins; a.min_area = p.min_area;
  a.ws = static_cast<char*>(p.ws);
  a.lay = layout(p.H, p.W, p.K, p.num_bins);
  a.records = p.records;
  // zero the per-frame counters and histograms (one contiguous, 256-B aligned region).
  // A kernel, not hipMemsetAsync: a memset node captured by torch.cuda.graph faulted
  // (illegal address) on its second replay on ROCm 7.x; kernel nodes replay cleanly.
  const size_t n16 = a.lay.small_bytes * p.B / 16;
  hipLaunchKernelGGL(k_zero, dim3((unsigned)std::min<size_t>((n16 + 255) / 256, 1024)), dim3(256), 0,
                     s, reinterpret_cast<uint4*>(a.ws), n16);
  const int N = p.crop_h * p.crop_w;
  const dim3 blk(256);
  const dim3 gp(cdiv(N, 256), p.B);
  const int Q = (p.crop_w - 1) * (p.crop_h - 1);
  const dim3 gq(cdiv(std::max(Q, 1), 256), p.B);
  // SSA_POST_STAGES=n (debug) launches only the first n stages
  static const int stages = [] {
    const char* e = getenv("SSA_POST_STAGES");
    return e ? atoi(e) : 99;
  }();
  int st = 0;
  const dim3 gt(cdiv(p.crop_w, TW), cdiv(p.crop_h, TH), p.B);
  if (st++ < stages) hipLaunchKernelGGL(k_ccl_local, gt, blk, 0, s, a, p.palette);
  if (st++ < stages) hipLaunchKernelGGL(k_ccl_boundary, gp, blk, 0, s, a);
  if (st++ < stages) hipLaunchKernelGGL(k_compress, gp, blk, 0, s, a);
  if (st++ < stages) hipLaunchKernelGGL(k_roots, gp, blk, 0, s, a);
  if (st++ < stages) hipLaunchKernelGGL(k_quads, gq, blk, 0, s, a);
  if (st++ < stages) hipLaunchKernelGGL(k_tree, gp, blk, 0, s, a);
  if (st++ < stages) hipLaunchKernelGGL(k_select, gp, blk, 0, s, a);
  if (st++ < stages) hipLaunchKernelGGL(k_hist, gp, blk, 0, s, a);
  if (st++ < stages) hipLaunchKernelGGL(k_finalize, dim3(p.B), dim3(64), 0, s, a);
  check_launch("postprocess");
}

}  // namespace ssa
