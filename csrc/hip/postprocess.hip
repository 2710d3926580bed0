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
//   k_ccl_local  per 32x32 tile: palette -> 3x3 box blur (REFLECT_101, rounded) ->
//                BGR2GRAY on RGB (fixed point) -> > thr, then union-find in LDS:
//                foreground 8-connected, background 4-connected; zeroes the counters
//   k_ccl_edges  cross-tile unions as pairs of tile-local roots (frames past kMergeCap
//                roots: applied to L right away, a global union-find)
//   k_ccl_merge  one workgroup per frame: union-find over those pairs in LDS;
//                image-border background joins the virtual "outside" node 0; final
//                labels of the tile-local roots (a label is an entry of the batch's root
//                pool + 1, 0 = outside); roots zero their accumulators. Extra workgroups
//                of the same grid relabel the union-find frames.
//   k_accum      per pixel: its 2x2 quad's polygon pieces as exact integer moments
//                (a00 = 2A, a10 = 6*int x, a01 = 6*int y) and its class into the fill
//                histograms (component + everything it encloses; holes also get the
//                parent's ring pixels), strip-privatised in LDS and added to every
//                ancestor in the border tree at flush time (subtree sums)
//   k_records    one workgroup per frame: contours whose polygon area >= min_area get
//                a record slot (bitonic sort of the passing roots), then majority
//                label, score, centroid (OpenCV's double arithmetic), normalisation,
//                records in findContours pre-order
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>

namespace ssa {
namespace {

struct FrameWS {
  int32_t* L;          // [N + 1] union-find labels (index 0 = outside)
  uint8_t* mask;       // [N] 1 = foreground
  int32_t* nslot;      // [0] selected, [1] contours dropped (> K passed), [2] cross-tile edges,
                       // [3] component roots listed (zeroed by k_ccl_local)
  int32_t* slot_node;  // [K]
  int32_t* cidx;       // [N] per tile-local root pixel: its compact index (k_ccl_local), after
                       //     k_ccl_merge its final label; per component root (fallback): its label
  int32_t* rootpix;    // [ntiles][kTileCap] raster index of each tile-local root (tile-local index
                       //     c < kTileCap; the rest go to rovf)
  int32_t* ntroot;     // [ntiles] tile-local roots per tile
  int32_t* rovf;       // [kMergeCap][2] (tile * kTileRoots + c, raster index) of roots past kTileCap
  int32_t* flag;       // [8]: [0] = 1 -> global union-find fallback, [1] = 1 -> root pool exhausted
                       //      (no records), [2] rovf entries (k_ccl_local -> k_ccl_merge, which
                       //      re-zeroes it), [3] the frame's first pool entry
  int32_t* edges;      // [ecap][2] cross-tile unions (tile-local roots as raster, -1 = outside); ecap =
                       //     3 per edge-line pixel, so the list never overflows
  // root pool, shared by the batch and indexed by component label - 1 (labels are pool
  // entries: a frame's components take one contiguous run of it)
  int32_t* pool;       // [0] entries taken this call (zeroed by k_ccl_local)
  int32_t* t00;        // [P] subtree 2*area
  long long* t10;      // [P] subtree 6 * int x
  long long* t01;      // [P] subtree 6 * int y
  int32_t* th;         // [P][bins] class histogram of the contour's fill
  int32_t* rpar;       // [P] border-tree parent (label, 0 = frame; fallback frames: raster root + 1)
  int32_t* rlist;      // [P] raster index of the component's root (first) pixel
  int fb;              // (kernels after k_ccl_merge) flag[0]
};

#ifndef SSA_CCL_TH
#define SSA_CCL_TH 32
#endif
constexpr int TW = 32, TH = SSA_CCL_TH;  // local CCL tile
constexpr int kMergeCap = 12288;     // tile-local roots the per-frame LDS merge handles
constexpr int kTileRoots = TW * TH;  // worst case roots per tile
constexpr int kTileCap = 64;         // roots per tile with a rootpix slot (the rest: rovf)
constexpr int kPoolPerFrame = 8192;  // root pool entries per frame of the batch (floor: N + 1)

// Workspace layout (round 5): per frame only what is per pixel (labels, mask,
// compact index) plus the bounded merge inputs; everything per component lives in ONE pool
// for the batch, indexed by label, of max(B * kPoolPerFrame, N + 1) + N / 2 + 1 entries. A frame's
// components take a contiguous run of it (k_ccl_merge: one atomicAdd of its component count;
// fallback frames reserve their tile-local root count, an upper bound). The floor of N + 1
// entries keeps any single frame exact (a frame has fewer components than pixels); a batch
// whose components overflow the pool flags the frames that did not fit (flag[1]: no records,
// count NaN; never on segmentation maps -- the bench frames have ~200 components each).
// Round 4 indexed every per-root array by raster index: 46 MB per 513^2 frame.
struct Layout {
  size_t N, K, bins, P, ntiles, ecap;
  size_t small_bytes;  // nslot(16) + slot_node, per frame (zeroed every call)
  size_t big_bytes;    // per frame
  size_t pool_bytes;   // per batch
  size_t total(int B) const { return (small_bytes + big_bytes) * (size_t)B + 256 + pool_bytes; }
};

__host__ __device__ inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

Layout layout(int B, int H, int W, int K, int bins) {
  Layout l;
  l.N = (size_t)H * W;
  l.K = K;
  l.bins = bins;
  // + N / 2 + 1 beyond the shared part: with the floor, two frames of ANY content (a
  // union-find fallback frame reserves its tile-local root count, at most ~N / 2: a
  // checkerboard's 4-connected background) fit beside the batch's typical ones (ADVICE r5:
  // two speckled frames in one batch could exhaust a pool of max(B * 8192, N + 1))
  l.P = std::max((size_t)B * kPoolPerFrame, l.N + 1) + l.N / 2 + 1;
  l.ntiles = (size_t)((W + TW - 1) / TW) * ((H + TH - 1) / TH);
  // k_ccl_edges' unions at the largest crop: <= 3 per pixel of a tile top row, 2 of a tile
  // left column, 1 of a right column or of the image border
  const size_t txn = (W + TW - 1) / TW, tyn = (H + TH - 1) / TH;
  l.ecap = (tyn - 1) * W * 3 + 2 * (size_t)W + (txn - 1) * H * 3 + 2 * (size_t)H;
  l.small_bytes = al(16 + (size_t)K * 4);
  l.big_bytes = al((l.N + 1) * 4) + al(l.N) + al(l.N * 4) + al(l.ntiles * kTileCap * 4) + al(l.ntiles * 4) +
                al((size_t)kMergeCap * 8) + al(32) + al(l.ecap * 8);
  l.pool_bytes = 2 * al(l.P * 8) + 3 * al(l.P * 4) + al(l.P * bins * 4);
  return l;
}

__host__ __device__ inline FrameWS frame_ws(char* ws, const Layout& l, int B, int b) {
  FrameWS f;
  char* s = ws + (size_t)b * l.small_bytes;
  f.nslot = reinterpret_cast<int32_t*>(s);
  f.slot_node = reinterpret_cast<int32_t*>(s + 16);
  char* hdr = ws + (size_t)B * l.small_bytes;
  f.pool = reinterpret_cast<int32_t*>(hdr);
  char* p = hdr + 256 + (size_t)b * l.big_bytes;
  f.L = reinterpret_cast<int32_t*>(p); p += al((l.N + 1) * 4);
  f.mask = reinterpret_cast<uint8_t*>(p); p += al(l.N);
  f.cidx = reinterpret_cast<int32_t*>(p); p += al(l.N * 4);
  f.rootpix = reinterpret_cast<int32_t*>(p); p += al(l.ntiles * kTileCap * 4);
  f.ntroot = reinterpret_cast<int32_t*>(p); p += al(l.ntiles * 4);
  f.rovf = reinterpret_cast<int32_t*>(p); p += al((size_t)kMergeCap * 8);
  f.flag = reinterpret_cast<int32_t*>(p); p += al(32);
  f.edges = reinterpret_cast<int32_t*>(p);
  char* q = hdr + 256 + (size_t)B * l.big_bytes;
  f.t10 = reinterpret_cast<long long*>(q); q += al(l.P * 8);
  f.t01 = reinterpret_cast<long long*>(q); q += al(l.P * 8);
  f.t00 = reinterpret_cast<int32_t*>(q); q += al(l.P * 4);
  f.rpar = reinterpret_cast<int32_t*>(q); q += al(l.P * 4);
  f.rlist = reinterpret_cast<int32_t*>(q); q += al(l.P * 4);
  f.th = reinterpret_cast<int32_t*>(q);
  f.fb = 0;
  return f;
}

struct KArgs {
  const uint8_t* labels;  // [B, H, W]
  int B, H, W, ch, cw, thr, K, bins;
  double min_area;
  char* ws;
  Layout lay;
  float* records;
  int dbg;  // SSA_POST_DBG ablation bits (timing experiments only; 0 in production)
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
// One 256-thread block = one TW x TH = 32 x 32 pixel tile, four pixels per thread
// (rows ty + 8k), half a wave per tile row.
//  1. mask: the tile's labels + 1-pixel REFLECT_101 halo are staged in LDS, the
//     palette colours are box-summed separably (horizontal 3-sums in LDS, then
//     vertical), rounded per channel like cv2.blur, converted with the fixed-point
//     BGR2GRAY weights and thresholded;
//  2. runs: each row's mask is one 32-bit ballot; a pixel's initial label is the
//     start of its horizontal run (foreground and background runs alike), so the
//     horizontal unions cost nothing;
//  3. the only unions are between a run and each run of the row above that it
//     touches (8-neighbourhood for foreground, 4 for background), one union per
//     touching pair, issued by the pixel where the overlap starts;
//  4. every root is the minimum tile index of its set (atomicMin linking), so the
//     global label (raster index + 1 of the tile-local root) keeps the global
//     min-root invariant the boundary merge relies on.
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

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// 256 threads per TW x TH tile: each thread owns RPT = TW * TH / 256 pixels of one
// column (rows ty + 8 k), so a block's global-load and barrier latency is paid once per
// RPT pixels (256 threads: 51 us per 32 bench frames vs 61 us at 512 and 94 us at 1024,
// profiles/r3_post_ab.txt), and the 32 x 32 tile keeps the cross-tile edges / tile-local
// roots the merge handles low.
#ifndef SSA_CCL_THREADS
#define SSA_CCL_THREADS 256
#endif
constexpr int kCclThreads = SSA_CCL_THREADS;
constexpr int RPT = TH * TW / kCclThreads;
static_assert(RPT * kCclThreads == TW * TH && TW == 32 && kCclThreads % 64 == 0, "k_ccl_local: 32-wide tiles");

__global__ __launch_bounds__(kCclThreads) void k_ccl_local(KArgs a, const int32_t* __restrict__ pal) {
  constexpr int HW2 = TW + 2, HH2 = TH + 2, RS = kCclThreads / TW;  // RS: row stride of a thread's pixels
  __shared__ int spal[256];  // packed r | g << 10 | b << 20 (3-sums of a field stay < 1024)
  __shared__ uint8_t slab[HH2 * HW2];
  __shared__ int hs[HH2 * TW];  // packed horizontal 3-sums
  __shared__ int lbl[TW * TH];
  __shared__ unsigned fgrow[TH], bgrow[TH];
  __shared__ int s_nroot;
  const int tid = threadIdx.x;
  if (tid == 0) s_nroot = 0;
  for (int i = tid; i < 256; i += kCclThreads)
    spal[i] = (pal[3 * i] & 255) | (pal[3 * i + 1] & 255) << 10 | (pal[3 * i + 2] & 255) << 20;
  const int b = blockIdx.z;
  const int x0 = blockIdx.x * TW, y0 = blockIdx.y * TH;
  const int tx = tid % TW, ty0 = tid / TW;
  const int x = x0 + tx;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) {
    f.L[0] = 0;
    if (b == 0) *f.pool = 0;  // read first by k_ccl_merge
  }
  {  // the frame's tiles zero its counters (round 2 spent a k_zero launch on this)
    uint4* z = reinterpret_cast<uint4*>(a.ws + (size_t)b * a.lay.small_bytes);
    const int words = (int)(a.lay.small_bytes / 16), nt = gridDim.x * gridDim.y;
    for (int i = (blockIdx.y * gridDim.x + blockIdx.x) * kCclThreads + tid; i < words; i += nt * kCclThreads)
      z[i] = make_uint4(0, 0, 0, 0);
  }
  const uint8_t* lab = a.labels + (size_t)b * a.H * a.W;
  for (int i = tid; i < HH2 * HW2; i += kCclThreads) {
    const int yy = clampi(reflect101(y0 - 1 + i / HW2, a.ch), 0, a.ch - 1);
    const int xx = clampi(reflect101(x0 - 1 + i % HW2, a.cw), 0, a.cw - 1);
    slab[i] = lab[yy * a.W + xx];
  }
  __syncthreads();
  for (int i = tid; i < HH2 * TW; i += kCclThreads) {
    const int r = i / TW, c = i % TW;
    const uint8_t* sr = slab + r * HW2 + c;
    const int l0 = sr[0], l1 = sr[1], l2 = sr[2];
    hs[i] = spal[l0] + spal[l1] + spal[l2];
  }
  __syncthreads();
  bool m[RPT], in[RPT];
  unsigned fgm[RPT], bgm[RPT];
  int start[RPT];
  const int half = (tid & 63) >> 5;
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int ty = ty0 + k * RS, y = y0 + ty;
    in[k] = x < a.cw && y < a.ch;
    m[k] = false;
    if (in[k]) {
      int c[3];
      const int h0 = hs[ty * TW + tx], h1 = hs[(ty + 1) * TW + tx], h2 = hs[(ty + 2) * TW + tx];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const int sum = ((h0 >> (10 * ch)) & 1023) + ((h1 >> (10 * ch)) & 1023) + ((h2 >> (10 * ch)) & 1023);
        c[ch] = (sum * 2 + 9) / 18;
      }
      const int g = (c[0] * 1868 + c[1] * 9617 + c[2] * 4899 + (1 << 13)) >> 14;
      m[k] = g > a.thr;
      f.mask[y * a.cw + x] = m[k] ? 1 : 0;
    }
    // per-row run bitmasks (bit = column); lanes 0-31 / 32-63 of a wave are two rows
    const unsigned long long bf = __ballot(in[k] && m[k]), bb = __ballot(in[k] && !m[k]);
    fgm[k] = (unsigned)(bf >> (32 * half));
    bgm[k] = (unsigned)(bb >> (32 * half));
    if ((tid & 31) == 0) {
      fgrow[ty] = fgm[k];
      bgrow[ty] = bgm[k];
    }
    const unsigned mine = m[k] ? fgm[k] : bgm[k];
    const int me = ty * TW + tx;
    start[k] = me;
    if (in[k]) {
      const unsigned starts = mine & ~(mine << 1);
      start[k] = ty * TW + 31 - __clz(starts & (0xffffffffu >> (31 - tx)));
    }
    lbl[me] = start[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int ty = ty0 + k * RS, me = ty * TW + tx;
    if (!in[k] || ty == 0) continue;
    const unsigned bit = 1u << tx;
    const int up = me - TW;
    if (m[k]) {
      const unsigned u = fgrow[ty - 1];
      const unsigned ends = fgm[k] & ~(fgm[k] >> 1);
      const bool first = (me == start[k]);
      const bool last = (ends & bit) != 0;
      if ((u & bit) && (first || !(u & (bit >> 1)))) lunite(lbl, start[k], up);
      if (first && tx > 0 && (u & (bit >> 1)) && !(u & bit)) lunite(lbl, start[k], up - 1);
      if (last && tx < 31 && (u & (bit << 1)) && !(u & bit)) lunite(lbl, start[k], up + 1);
    } else {
      const unsigned u = bgrow[ty - 1];
      if ((u & bit) && (me == start[k] || !(u & (bit >> 1)))) lunite(lbl, start[k], up);
    }
  }
  __syncthreads();
  const int tile = blockIdx.y * gridDim.x + blockIdx.x;
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int ty = ty0 + k * RS, y = y0 + ty, me = ty * TW + tx;
    if (!in[k]) continue;
    const int r = lfind(lbl, start[k]);
    const int rx = x0 + r % TW, ry = y0 + r / TW;
    f.L[y * a.cw + x + 1] = ry * a.cw + rx + 1;
    if (r == me) {  // tile-local root: numbered within the tile (k_ccl_merge scans the counts)
      const int c = atomicAdd(&s_nroot, 1);
      f.cidx[y * a.cw + x] = c;
      if (c < kTileCap) {
        f.rootpix[tile * kTileCap + c] = y * a.cw + x;
      } else {  // a crowded tile: listed (rare; at most kMergeCap of them matter)
        const int o = atomicAdd(f.flag + 2, 1);
        if (o < kMergeCap) {
          f.rovf[2 * o] = tile * kTileRoots + c;
          f.rovf[2 * o + 1] = y * a.cw + x;
        }
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    f.ntroot[tile] = s_nroot;
    atomicAdd(f.flag + 4, s_nroot);  // the frame's root count (k_ccl_edges decides the path)
  }
}

// ---------------------------------------------------------------- compact merge
// Cross-tile merging in two steps.
// k_ccl_edges: every pixel on a tile edge (or on the image border) emits the
//   unions it needs as pairs of tile-local roots (-1 = the outside node). Lanes
//   run along the edge (x for horizontal edges, y for vertical ones), so the
//   long runs of identical pairs a blob produces collapse to one pair with a
//   compare against the previous lane; survivors are appended with one atomic
//   per wave.
// k_ccl_merge: ONE workgroup per frame numbers the tile-local roots (a few per
//   tile on real masks) compactly, runs union-find over the pair list on LDS
//   atomics, writes every tile-local root's final label (min raster index + 1,
//   outside-connected background -> 0) over its cidx entry, zeroes the accumulators
//   of every component root and lists the roots. Pixels are resolved on the fly
//   afterwards (fin(): L -> tile-local root -> cidx): no full-frame relabelling pass
//   (round 2's k_compress, 22 us per 32 frames).
// Frames past kMergeCap roots take the global union-find (device-coherent pointer chasing)
// across the tile edges inside k_ccl_edges and a relabelling pass in the merge grid (see
// fb_relabel); fin() reads the same two levels (L -> root -> cidx) for both.
// wave-aggregated append of this lane's kept pairs (me, o0..o2; k0..k2 = kept)
__device__ __forceinline__ void emit_pairs(FrameWS& f, size_t ecap, int me, int o0, int o1, int o2, bool k0, bool k1,
                                           bool k2) {
  const int n = (int)k0 + (int)k1 + (int)k2;
  int incl = n;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const int total = __shfl(incl, 63, 64);
  if (total == 0) return;
  int base = 0;
  if (lane == 63) base = atomicAdd(f.nslot + 2, total);
  base = __shfl(base, 63, 64);
  int at = base + incl - n;
  auto put = [&](int o) {
    if (at < (int)ecap) {  // (never false: ecap covers 3 unions per line pixel)
      f.edges[2 * at] = me;
      f.edges[2 * at + 1] = o;
    }
    ++at;
  };
  if (k0) put(o0);
  if (k1) put(o1);
  if (k2) put(o2);
}

constexpr int kEdgeThreads = 256;

__global__ __launch_bounds__(kEdgeThreads) void k_ccl_edges(KArgs a) {
  const int b = blockIdx.z;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  // frames past kMergeCap tile-local roots take the global union-find right here: the
  // same unions, applied to L (device-coherent pointer chasing) instead of listed; one
  // thread per frame reserves their root count (>= the components) from the pool
  const int R = __builtin_amdgcn_readfirstlane(f.flag[4]);
  const bool fb = R > kMergeCap;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    f.flag[0] = fb ? 1 : 0;
    if (fb) {
      const int base = atomicAdd(f.pool, R);
      f.flag[1] = (size_t)base + R > a.lay.P ? 1 : 0;
      f.flag[3] = base;
    }
  }
  const int tx_n = (a.cw + TW - 1) / TW, ty_n = (a.ch + TH - 1) / TH;
  // horizontal lines: tile top rows y = k*TH (k >= 1), image rows 0 and ch-1;
  // vertical lines: tile left columns x = k*TW (k >= 1), right columns x = k*TW-1
  // (k >= 1, x < cw-1), image columns 0 and cw-1
  const int nh = (ty_n - 1) + 2, nv = 2 * (tx_n - 1) + 2;
  const int line = blockIdx.y;
  const bool horiz = line < nh;
  int fixed, len;
  int kind;  // 0 top row, 1 border row, 2 left column, 3 right column, 4 border column
  if (horiz) {
    if (line < ty_n - 1) { fixed = (line + 1) * TH; kind = 0; }
    else { fixed = line == ty_n - 1 ? 0 : a.ch - 1; kind = 1; }
    len = a.cw;
  } else {
    const int l = line - nh;
    if (l >= nv) return;
    if (l < tx_n - 1) { fixed = (l + 1) * TW; kind = 2; }
    else if (l < 2 * (tx_n - 1)) { fixed = (l - (tx_n - 1) + 1) * TW - 1; kind = 3; }
    else { fixed = l == 2 * (tx_n - 1) ? 0 : a.cw - 1; kind = 4; }
    len = a.ch;
  }
  // (one 192-thread block per line, looping over the line, measured 2 us slower than a
  // block per 256 pixels: profiles/r3_post_ab.txt)
  for (int i0 = blockIdx.x * blockDim.x; i0 < len; i0 += gridDim.x * blockDim.x) {
    const int i = i0 + (int)threadIdx.x;
    const bool valid = i < len && fixed >= 0 && (horiz ? fixed < a.ch : fixed < a.cw) &&
                       !(kind == 3 && fixed + 1 >= a.cw);
    const int x = horiz ? i : fixed, y = horiz ? fixed : i;
    const int p = y * a.cw + x;
    // up to three partners of this pixel's tile-local root across the edge (-2 = none)
    int me = -2, o0 = -2, o1 = -2, o2 = -2;
    if (valid) {
      const bool m = f.mask[p] != 0;
      me = f.L[p + 1] - 1;
      auto lr = [&](int q) { return f.L[q + 1] - 1; };
      if (kind == 0) {  // top row of a tile: unions with the row above
        const int up = p - a.cw;
        if (m) {
          if (x > 0 && f.mask[up - 1]) o0 = lr(up - 1);
          if (f.mask[up]) o1 = lr(up);
          if (x + 1 < a.cw && f.mask[up + 1]) o2 = lr(up + 1);
        } else if (!f.mask[up]) {
          o0 = lr(up);
        }
      } else if (kind == 2) {  // left column of a tile: unions with the column to the left
        if (m) {
          if (f.mask[p - 1]) o0 = lr(p - 1);
          if (y > 0 && (y % TH) != 0 && f.mask[p - a.cw - 1]) o1 = lr(p - a.cw - 1);
        } else if (!f.mask[p - 1]) {
          o0 = lr(p - 1);
        }
      } else if (kind == 3) {  // right column: up-right diagonal into the next tile
        if (m && y > 0 && (y % TH) != 0 && f.mask[p - a.cw + 1]) o0 = lr(p - a.cw + 1);
      }
      if ((kind == 1 || kind == 4) && !m) o0 = -1;  // image-border background -> outside
    }
    // distinct partners only, and drop pairs the previous lane (previous pixel along this
    // line) also emitted
    const int lane = threadIdx.x & 63;
    const int pm = __shfl_up(me, 1, 64);
    const int p0 = __shfl_up(o0, 1, 64), p1 = __shfl_up(o1, 1, 64), p2 = __shfl_up(o2, 1, 64);
    auto seen = [&](int o) { return lane > 0 && pm == me && (o == p0 || o == p1 || o == p2); };
    const bool k0 = o0 != -2 && !seen(o0);
    const bool k1 = o1 != -2 && o1 != o0 && !seen(o1);
    const bool k2 = o2 != -2 && o2 != o0 && o2 != o1 && !seen(o2);
    if (fb) {
      if (k0) unite(f.L, me + 1, o0 + 1);  // (-1 + 1 = the outside node 0)
      if (k1) unite(f.L, me + 1, o1 + 1);
      if (k2) unite(f.L, me + 1, o2 + 1);
    } else {
      emit_pairs(f, a.lay.ecap, me, o0, o1, o2, k0, k1, k2);
    }
  }
}

// A component root takes pool entry n (label n + 1): its accumulators zeroed, listed
__device__ __forceinline__ void new_root(FrameWS& f, int bins, int n, int p) {
  f.t00[n] = 0;
  f.t10[n] = 0;
  f.t01[n] = 0;
  int* h = f.th + (size_t)n * bins;
  for (int c = 0; c < bins; ++c) h[c] = 0;
  f.rlist[n] = p;
}

__device__ void fb_relabel(const KArgs& a, int bi, int nb);

__global__ __launch_bounds__(1024) void k_ccl_merge(KArgs a) {
  extern __shared__ int sm[];
  if ((int)blockIdx.x >= a.B) {  // the union-find frames' relabel (idle unless one is flagged)
    fb_relabel(a, blockIdx.x - a.B, gridDim.x - a.B);
    return;
  }
  const int b = blockIdx.x;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  const int cw = a.cw, ch = a.ch;
  const int tx_n = (cw + TW - 1) / TW, ty_n = (ch + TH - 1) / TH;
  const int nt = tx_n * ty_n;
  const int tid = threadIdx.x;
  int* par = sm;                    // [kMergeCap + 1] (last = outside)
  int* minr = par + kMergeCap + 1;  // [kMergeCap + 1] set minimum pixel, then the set's label
  int* rp = minr + kMergeCap + 1;   // [kMergeCap] raster index of compact root i
  int* toff = rp + kMergeCap;       // [nt + 1]
  int* part = toff + nt + 1;        // [1024] scan partials
  int* s_c = part + 1024;           // [0] components, [1] listed, [2] pool base (-1: exhausted)
  if (tid == 0) { s_c[0] = 0; s_c[1] = 0; }
  // exclusive scan of the per-tile root counts: compact index = tile offset + tile-local index
  const int per = (nt + 1023) / 1024;
  const int t0 = tid * per, t1 = min(nt, t0 + per);
  int sum = 0;
  for (int t = t0; t < t1; ++t) sum += f.ntroot[t];
  part[tid] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int acc = part[tid] - sum;
  for (int t = t0; t < t1; ++t) {
    toff[t] = acc;
    acc += f.ntroot[t];
  }
  if (tid == 1023) toff[nt] = part[1023];
  __syncthreads();
  const int R = toff[nt];
  const int E = f.nslot[2];
  const int O = f.flag[2];
  __syncthreads();
  if (tid == 0) {  // k_ccl_local's counters, read (here and by k_ccl_edges) for this call
    f.flag[2] = 0;
    f.flag[4] = 0;
  }
  if (R > kMergeCap) return;  // k_ccl_edges united it in L and took its pool run; the relabel
                              // blocks of this grid label it
  const int OUT = R;
  auto tile_of = [&](int i) {  // last tile t with toff[t] <= i (empty tiles share offsets)
    int lo = 0, hi = nt - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (toff[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  for (int i = tid; i <= R; i += 1024) {
    par[i] = i;
    minr[i] = 0x7fffffff;
    if (i < R) {
      const int t = tile_of(i), c = i - toff[t];
      if (c < kTileCap) rp[i] = f.rootpix[t * kTileCap + c];
    }
  }
  for (int o = tid; o < O; o += 1024) {
    const int key = f.rovf[2 * o], t = key / kTileRoots;
    rp[toff[t] + key - t * kTileRoots] = f.rovf[2 * o + 1];
  }
  __syncthreads();
  auto compact = [&](int r) {
    const int ly = r / cw, lx = r - ly * cw;
    return toff[(ly / TH) * tx_n + lx / TW] + f.cidx[r];
  };
  for (int e = tid; e < E; e += 1024) {
    const int ra = f.edges[2 * e], rb = f.edges[2 * e + 1];
    lunite(par, compact(ra), rb < 0 ? OUT : compact(rb));
  }
  __syncthreads();
  for (int i = tid; i < R; i += 1024) atomicMin(&minr[lfind(par, i)], rp[i]);
  __syncthreads();
  const int outroot = lfind(par, OUT);
  // every set but the outside one is a component: count, take a run of the pool, list
  for (int i = tid; i < R; i += 1024)
    if (i != outroot && par[i] == i) atomicAdd(s_c, 1);
  __syncthreads();
  if (tid == 0) {
    const int nr = s_c[0];
    const int base = atomicAdd(f.pool, nr);
    const bool ex = (size_t)base + nr > a.lay.P;
    s_c[2] = ex ? -1 : base;
    f.flag[1] = ex ? 1 : 0;
    f.flag[3] = base;
    f.nslot[3] = nr;
  }
  __syncthreads();
  const int base = s_c[2];
  if (base < 0) return;
  for (int i = tid; i < R; i += 1024) {
    if (i != outroot && par[i] == i) {
      const int n = base + atomicAdd(s_c + 1, 1);
      new_root(f, a.bins, n, minr[i]);  // the root: the component's minimum pixel
      minr[i] = n + 1;
    }
  }
  __syncthreads();
  // final label of every tile-local root, over its cidx entry (the compact indices are done)
  for (int i = tid; i < R; i += 1024) {
    const int r = lfind(par, i);
    f.cidx[rp[i]] = r == outroot ? 0 : minr[r];
  }
  __syncthreads();
  // border-tree parent of every root: the final label of the pixel left of it
  const int nr = s_c[0];
  for (int j = tid; j < nr; j += 1024) {
    const int p = f.rlist[base + j];
    f.rpar[base + j] = p % cw > 0 ? f.cidx[f.L[p] - 1] : 0;
  }
}

// Fallback for frames past the LDS merge's cap (more than kMergeCap tile-local roots:
// speckled maps). Round 3 ran it inside one k_ccl_merge workgroup per frame: 813 us for a
// frame of ~12k components (the lattice maps of csrc/tools/post_bench.hip).
// Since round 5 it costs no launch of its own: k_ccl_edges applies the frame's cross-tile
// unions to L directly (global union-find), and extra workgroups of the k_ccl_merge grid
// relabel it (every pixel's root, read-only traversal: concurrent stores only ever write
// roots), zero and list the roots' pool entries, and record each root's border-tree parent
// (the root of the pixel left of it, by the same traversal). Round 4 spent two grid
// launches (k_fb_unite, k_fb_relabel) on this: ~11 us per step of no-ops in the step trace;
// a separate small relabel grid read 11-21 us there (profiles/r5z_layer_times.txt).
constexpr int kFbBlocks = 64;  // relabel workgroups of the merge grid (grid-stride per frame)

// The flagged frames of the batch, as a bitmask per 64 frames (every wave of the block
// computes the same mask from the same flags; one load per lane, not a chain of B loads).
__device__ __forceinline__ unsigned long long fb_frames(const KArgs& a, int b0) {
  const int b = b0 + (int)(threadIdx.x & 63);
  bool need = false;
  if (b < a.B) {
    const FrameWS g = frame_ws(a.ws, a.lay, a.B, b);
    need = g.flag[0] != 0 && g.flag[1] == 0;
  }
  return __ballot(need);
}

__device__ void fb_relabel(const KArgs& a, int bi, int nb) {
  const int N = a.ch * a.cw, nt = blockDim.x;
  for (int b0 = 0; b0 < a.B; b0 += 64) {
    for (unsigned long long m = fb_frames(a, b0); m; m &= m - 1) {
      FrameWS f = frame_ws(a.ws, a.lay, a.B, b0 + __ffsll((long long)m) - 1);
      const int base = f.flag[3];
      for (int p = bi * nt + threadIdx.x; p < N; p += nb * nt) {
        const int r = find_root(f.L, p + 1);
        __hip_atomic_store(f.L + p + 1, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (r == p + 1) {
          const int n = base + atomicAdd(f.nslot + 3, 1);  // nslot[3] zeroed by k_ccl_local
          new_root(f, a.bins, n, p);
          f.rpar[n] = p % a.cw > 0 ? find_root(f.L, p) : 0;  // raster root + 1: parent_of maps it
          f.cidx[p] = n + 1;
        }
      }
    }
  }
}

// Parent of component n in the border tree: the component of the pixel left of its
// first pixel (0 = the frame at the image border), a pure function of the final labels,
// tabulated per root by k_ccl_merge (one load instead of the L -> cidx chain).
// Final component label of pixel q (root raster index + 1, 0 = outside).
// (L holds the tile-local root, or after the fallback the component root / 0 = outside;
// cidx of either is the label.)
__device__ __forceinline__ int fin(const FrameWS& f, int q) {
  const int l = f.L[q + 1];
  return l == 0 ? 0 : f.cidx[l - 1];
}

__device__ __forceinline__ int parent_of(const FrameWS& f, int cw, int n) {
  const int r = f.rpar[n - 1];
  return (f.fb && r != 0) ? f.cidx[r - 1] : r;
}

// Per-block privatisation of the component sums. A real scene's mask has a few
// large components, so every quad of a blob adds into the same three global
// counters: same-address atomics serialise at one L2 channel (the atomic version
// of this pass took 127 us per 32 frames on calibrated masks). Each block owns a
// contiguous strip of quads (a few image rows: few distinct components), sums
// them in a small LDS open-addressing table keyed by component id, and flushes
// one global atomic per (block, component). A wave whose 64 lanes hit the same
// component is reduced by shuffles first; a full table falls back to global
// atomics, so correctness never depends on the table size.
#ifndef SSA_KHASH
#define SSA_KHASH 128  // 64 / 256 (with a 512 histogram table) measured equal / 5 us slower
#endif
constexpr int kHash = SSA_KHASH;  // per-block moments table (power of 2)
constexpr int kQuadBlocks = 192;  // target blocks per frame of the accumulation pass (4 rounds of 256 px at 513 x 385: 229 vs 244 us at 3 rounds, 329 at 1; profiles/r3_post_ab.txt)

struct QuadTable {
  int key[kHash];
  int s00[kHash];
  unsigned long long s10[kHash];
  unsigned long long s01[kHash];
};

// Subtree sums without a tree pass: every (block, component) partial is added to the
// component and all its ancestors at flush time (round 2 summed own pieces first and
// walked the ancestors per root in a separate full-frame pass, k_tree).
__device__ void moments_up(FrameWS& f, int cw, int node, int d00, long long d10, long long d01, int maxd) {
  for (int n = node, depth = 0; n != 0 && depth <= maxd; ++depth, n = parent_of(f, cw, n)) {
    atomicAdd(f.t00 + n - 1, d00);
    atomicAdd(reinterpret_cast<unsigned long long*>(f.t10 + n - 1), (unsigned long long)d10);
    atomicAdd(reinterpret_cast<unsigned long long*>(f.t01 + n - 1), (unsigned long long)d01);
  }
}

// Histogram keys: (node * bins + class) * 2 + ring (> 0 for node >= 1; 0 = empty slot).
// An own-pixel count goes to the node and all its ancestors (a contour's fill is its
// component plus everything it encloses); a ring count (parent pixels 4-adjacent to a
// hole, part of the hole contour's fill only) goes to the hole alone.
__device__ void hist_up(FrameWS& f, int cw, int bins, int key, int cnt, int maxd) {
  const int v = key >> 1, node = v / bins, c = v - node * bins;
  if (key & 1) {
    atomicAdd(f.th + (size_t)(node - 1) * bins + c, cnt);
    return;
  }
  for (int n = node, depth = 0; n != 0 && depth <= maxd; ++depth, n = parent_of(f, cw, n))
    atomicAdd(f.th + (size_t)(n - 1) * bins + c, cnt);
}

#ifndef SSA_KHHASH
#define SSA_KHHASH 256
#endif
constexpr int kHistHash = SSA_KHHASH;  // per-block histogram table (power of 2)

struct AccTable {
  int maxd;  // ancestor levels a flush adds to (65536; 0 = SSA_POST_DBG bit 4 timing ablation)
  QuadTable q;
  int hkey[kHistHash];
  int hcnt[kHistHash];
};

__device__ __forceinline__ void table_add(AccTable& T, FrameWS& f, int cw, int node, int d00,
                                          long long d10, long long d01) {
  int h = (int)(((unsigned)node * 2654435761u) >> 25) & (kHash - 1);
#pragma unroll 1
  for (int probe = 0; probe < 16; ++probe, h = (h + 1) & (kHash - 1)) {
    int k = __hip_atomic_load(&T.q.key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k == 0) {
      k = atomicCAS(&T.q.key[h], 0, node);
      if (k == 0) k = node;
    }
    if (k == node) {
      atomicAdd(&T.q.s00[h], d00);
      atomicAdd(&T.q.s10[h], (unsigned long long)d10);
      atomicAdd(&T.q.s01[h], (unsigned long long)d01);
      return;
    }
  }
  moments_up(f, cw, node, d00, d10, d01, T.maxd);
}

__device__ __forceinline__ void agg_add(AccTable& T, FrameWS& f, int cw, int node, int d00, long long d10,
                                        long long d01) {
  const bool active = node > 0;
  const unsigned long long act = __ballot(active);
  if (act == 0) return;
  const int leader = __ffsll((long long)act) - 1;
  const int lnode = __shfl(node, leader, 64);
  if (__all(!active || node == lnode)) {
    // one quad's pieces are < 2^19 (6x + 3, x < 65536), so a 64-lane sum fits in
    // 32 bits: reduce in int32 (half the cross-lane traffic of the 64-bit sums)
    int s00 = active ? d00 : 0;
    int s10 = active ? (int)d10 : 0, s01 = active ? (int)d01 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s00 += __shfl_xor(s00, o, 64);
      s10 += __shfl_xor(s10, o, 64);
      s01 += __shfl_xor(s01, o, 64);
    }
    if ((int)(threadIdx.x & 63) == leader) table_add(T, f, cw, lnode, s00, s10, s01);
  } else if (active) {
    table_add(T, f, cw, node, d00, d10, d01);
  }
}

__device__ __forceinline__ void htable_add(AccTable& T, FrameWS& f, int cw, int bins, int key, int cnt) {
  int h = (int)(((unsigned)key * 2654435761u) >> 24) & (kHistHash - 1);
#pragma unroll 1
  for (int probe = 0; probe < 16; ++probe, h = (h + 1) & (kHistHash - 1)) {
    int k = __hip_atomic_load(&T.hkey[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k == 0) {
      k = atomicCAS(&T.hkey[h], 0, key);
      if (k == 0) k = key;
    }
    if (k == key) {
      atomicAdd(&T.hcnt[h], cnt);
      return;
    }
  }
  hist_up(f, cw, bins, key, cnt, T.maxd);
}

// Wave-aggregated histogram add: the wave's lanes are grouped by key (one ballot per
// distinct key; class maps are blobby, so 64 consecutive pixels carry 1-4 distinct
// keys) and ONE lane per group adds the group's count.
__device__ __forceinline__ void hagg(AccTable& T, FrameWS& f, int cw, int bins, int key) {
  unsigned long long act = __ballot(key > 0);
  const int me = (int)(threadIdx.x & 63);
  while (act) {  // wave-uniform loop, at most 64 iterations
    const int leader = __ffsll((long long)act) - 1;
    const int lkey = __shfl(key, leader, 64);
    const unsigned long long grp = __ballot(key == lkey) & act;
    if (me == leader) htable_add(T, f, cw, bins, lkey, __popcll(grp));
    act &= ~grp;
  }
}

// ---------------------------------------------------------------- accumulate
// One pass over the frame's pixels, strip-privatised per block, producing everything
// k_records needs for every component:
//  * the 2x2 quad whose top-left corner is the pixel: polygon pieces (full square /
//    triangle) as exact integer moments a00 = 2A, a10 = 6*int x, a01 = 6*int y
//    (corner order TL, TR, BL, BR; triangle of corner k = k + its two quad neighbours,
//    sums of its 3 vertices' coordinates = 3x + TX[k], 3y + TY[k]);
//  * the pixel's class into its component's fill histogram, and into the ring
//    histogram of each distinct hole it is 4-adjacent to (holes of its own component).
// Round 2 ran this as three passes (k_quads, k_tree, k_hist: 92 us per 32 frames).
#ifndef SSA_ACC_THREADS
#define SSA_ACC_THREADS 256
#endif
constexpr int kAccThreads = SSA_ACC_THREADS;
static_assert(kAccThreads >= 64 && kAccThreads <= 256 && 256 % kAccThreads == 0,
              "k_accum: 64, 128 or 256 threads (the strip grid is counted in 256-pixel rounds)");

__global__ __launch_bounds__(kAccThreads) void k_accum(KArgs a) {
  __shared__ AccTable T;
  const int b = blockIdx.y;
  const int cw = a.cw, ch = a.ch, bins = a.bins;
  const int N = cw * ch;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  if (f.flag[1]) return;  // root pool exhausted: no records for this frame
  f.fb = f.flag[0];
  for (int i = threadIdx.x; i < kHash; i += kAccThreads) {
    T.q.key[i] = 0; T.q.s00[i] = 0; T.q.s10[i] = 0; T.q.s01[i] = 0;
  }
  for (int i = threadIdx.x; i < kHistHash; i += kAccThreads) {
    T.hkey[i] = 0; T.hcnt[i] = 0;
  }
  if (threadIdx.x == 0) T.maxd = (a.dbg & 4) ? 0 : 65536;
  __syncthreads();
  const uint8_t* lab = a.labels + (size_t)b * a.H * a.W;
  const int per = (N + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(N, p0 + per);
  for (int pb = p0; pb < p1; pb += kAccThreads) {
    const int p = pb + threadIdx.x;
    int fnode = 0, f00 = 0;
    long long f10 = 0, f01 = 0;
    int bn[2] = {0, 0}, b00[2] = {0, 0};
    long long b10[2] = {0, 0}, b01[2] = {0, 0};
    int hkey = 0, rkey[4] = {0, 0, 0, 0};
    // each lane loads its pixel and the one below; the quad's right column comes from
    // the next lane (consecutive pixels), so every label is resolved twice instead of
    // four times (the dependent L -> cidx loads are this pass's latency chain)
    const int lane = threadIdx.x & 63;
    int y = 0, x = 0, n0 = 0, n2 = 0;
    bool m0 = false, m2 = false;
    if (p < N) {
      y = p / cw;
      x = p - y * cw;
      m0 = f.mask[p] != 0;
      n0 = fin(f, p);
      if (y + 1 < ch) {
        m2 = f.mask[p + cw] != 0;
        n2 = fin(f, p + cw);
      }
    }
    bool m1 = __shfl_down((int)m0, 1, 64) != 0, m3 = __shfl_down((int)m2, 1, 64) != 0;
    int n1 = __shfl_down(n0, 1, 64), n3 = __shfl_down(n2, 1, 64);
    if (lane == 63 && p < N && x + 1 < cw) {
      m1 = f.mask[p + 1] != 0;
      n1 = fin(f, p + 1);
      if (y + 1 < ch) {
        m3 = f.mask[p + cw + 1] != 0;
        n3 = fin(f, p + cw + 1);
      }
    }
    if (p < p1) {
      const bool fgp = m0;
      const int np = n0;
      int c = lab[y * a.W + x];
      if (c >= bins) c = bins - 1;
      if (np != 0 && !(a.dbg & 1)) hkey = (np * bins + c) * 2;
      if (x + 1 < cw && y + 1 < ch) {
        const int TX[4] = {1, 2, 1, 2}, TY[4] = {1, 1, 2, 2};
        const int node[4] = {n0, n1, n2, n3};
        const bool fg[4] = {m0, m1, m2, m3};
        int nf = 0, missing = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
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
      // ring: the foreground pixels 4-adjacent to a hole that belong to the hole's parent
      // component are part of the hole contour's fill. Counted from the hole side (hole
      // pixels are rare; round-2's check from every foreground pixel cost ~20 us per 32
      // frames): a hole pixel credits each such neighbour r whose first 4-neighbour
      // (order left, right, up, down) inside the hole is this pixel, so r counts once.
      if (!fgp && np != 0 && !(a.dbg & 2)) {
        const int nbr[4] = {x > 0 ? p - 1 : -1, x + 1 < cw ? p + 1 : -1, y > 0 ? p - cw : -1,
                            y + 1 < ch ? p + cw : -1};
        bool fgn[4], any = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          fgn[k] = nbr[k] >= 0 && f.mask[nbr[k]];
          any |= fgn[k];
        }
        if (any) {  // interior hole pixels stop at the mask loads
          const int par = parent_of(f, cw, np);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (!fgn[k]) continue;
            const int r = nbr[k];
            const int ry = r / cw, rx = r - ry * cw;
            // r's 4-neighbours that precede this pixel in r's (left, right, up, down) order:
            // this pixel is r's right (k = 0), left (k = 1), down (k = 2) or up (k = 3)
            // neighbour; their labels are loaded together, not in a chain
            int pre[3] = {-1, -1, -1};
            if (k == 0) {
              pre[0] = rx > 0 ? r - 1 : -1;
            } else if (k == 2) {
              pre[0] = rx > 0 ? r - 1 : -1;
              pre[1] = rx + 1 < cw ? r + 1 : -1;
              pre[2] = ry > 0 ? r - cw : -1;
            } else if (k == 3) {
              pre[0] = rx > 0 ? r - 1 : -1;
              pre[1] = rx + 1 < cw ? r + 1 : -1;
            }
            const int fr = fin(f, r);
            bool first = true;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              const int q = pre[j];
              if (q >= 0 && !f.mask[q] && fin(f, q) == np) first = false;
            }
            if (fr != par || !first) continue;
            int rc = lab[ry * a.W + rx];
            if (rc >= bins) rc = bins - 1;
            rkey[k] = (np * bins + rc) * 2 + 1;
          }
        }
      }
    }
    agg_add(T, f, cw, fnode, f00, f10, f01);
    agg_add(T, f, cw, bn[0], b00[0], b10[0], b01[0]);
    agg_add(T, f, cw, bn[1], b00[1], b10[1], b01[1]);
    hagg(T, f, cw, bins, hkey);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (__any(rkey[k] > 0)) hagg(T, f, cw, bins, rkey[k]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHash; i += kAccThreads) {
    const int node = T.q.key[i];
    if (node != 0) moments_up(f, cw, node, T.q.s00[i], (long long)T.q.s10[i], (long long)T.q.s01[i], T.maxd);
  }
  for (int i = threadIdx.x; i < kHistHash; i += kAccThreads) {
    const int key = T.hkey[i];
    if (key != 0) hist_up(f, cw, bins, key, T.hcnt[i], T.maxd);
  }
}

// Tile variant of k_accum (round 4; round 5 tables): one 256-thread block per AT x AT tile
// of a frame. The strip kernel resolves every label it touches through the dependent global
// chain L -> tile-local root -> cidx (fin()), per 256-pixel round; here the block stages the
// final labels, the mask and the classes of its tile plus the halo the per-pixel logic reads
// (2 columns left / right, 2 rows above, 1 below) in LDS first -- every global load of the
// chain issued at once, one round trip per chain level for the whole tile -- and the
// per-pixel logic below is k_accum's, reading LDS: same pieces, same sums.
// Round 5 (ablations on the bench model's own label maps, profiles/r5n_post_ablation.txt:
// moments 29 us, flush 19 us, class histogram 13 us, hole rings 10 us of 83 us per 32
// frames): the block's components get SLOTS of one small table (key = label); moments are
// wave-summed with DPP row adds + 4 readlanes (no ds_bpermute chains) and added to the slot;
// class counts go to a dense [slot][class] LDS counter (own pixels in the low 16 bits, hole
// rings in the high 16: no (node, class) hash probing, one single-lane atomic per distinct
// class of a node-uniform wave); the flush walks each slot's border-tree ancestors ONCE
// (one lane per slot, cached in LDS) and then issues only fire-and-forget atomics.
constexpr int kTSlots = 64;      // components per block in the table (more: global atomics)
constexpr int kDenseBins = 32;   // dense class counters per slot (bins <= 32; else k_accum)
constexpr int kAnc = 8;          // ancestors cached per slot

struct TileAcc {
  int key[kTSlots];  // component label, 0 = free
  int s00[kTSlots];
  unsigned s10[kTSlots], s01[kTSlots];  // a tile's sums stay < 2^31 (<= 4096 quads x 6x+3, x < 65536)
  int hist[kTSlots * kDenseBins];  // own count | ring count << 16 (both < 2^16 per tile)
  int anc[kTSlots][kAnc];
  int nanc[kTSlots], deep[kTSlots];
};

// Sum over the 64 lanes (all lanes active): quad and row butterflies in DPP, then the four
// row sums by readlane (wave-uniform result).
__device__ __forceinline__ int wave_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
         __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}

// slot of component `node` (inserted if new), -1 if the table's probe window is full
__device__ __forceinline__ int tslot(TileAcc& T, int node) {
  int h = (int)(((unsigned)node * 2654435761u) >> 26) & (kTSlots - 1);
#pragma unroll 1
  for (int probe = 0; probe < 16; ++probe, h = (h + 1) & (kTSlots - 1)) {
    int k = __hip_atomic_load(&T.key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k == 0) k = atomicCAS(&T.key[h], 0, node);
    if (k == 0 || k == node) return h;
  }
  return -1;
}

__device__ __forceinline__ void tmom(TileAcc& T, FrameWS& f, int cw, int node, int d00, int d10, int d01) {
  const int h = tslot(T, node);
  if (h < 0) {
    moments_up(f, cw, node, d00, d10, d01, 65536);
    return;
  }
  atomicAdd(&T.s00[h], d00);
  atomicAdd(&T.s10[h], (unsigned)d10);
  atomicAdd(&T.s01[h], (unsigned)d01);
}

// wave-aggregated moments piece (node 0 = none); wave-uniform control flow
__device__ __forceinline__ void tagg(TileAcc& T, FrameWS& f, int cw, int node, int d00, int d10, int d01) {
  const unsigned long long act = __ballot(node > 0);
  if (act == 0) return;
  const int leader = __ffsll((long long)act) - 1;
  const int lnode = __builtin_amdgcn_readlane(node, leader);
  if (__all(node <= 0 || node == lnode)) {
    // one quad's pieces are < 2^19 (6x + 3, x < 65536): a 64-lane sum fits in 32 bits
    const bool on = node > 0;
    const int s00 = wave_sum(on ? d00 : 0), s10 = wave_sum(on ? d10 : 0), s01 = wave_sum(on ? d01 : 0);
    if ((int)(threadIdx.x & 63) == leader) tmom(T, f, cw, lnode, s00, s10, s01);
  } else if (node > 0) {
    tmom(T, f, cw, node, d00, d10, d01);
  }
}

// global class count (table full): own counts up the ancestors, ring counts to the node
__device__ __forceinline__ void hist_global(FrameWS& f, int cw, int bins, int node, int c, int cnt, bool ring) {
  hist_up(f, cw, bins, (node * bins + c) * 2 + (ring ? 1 : 0), cnt, 65536);
}

template <int AT>
__global__ __launch_bounds__(256) void k_accum_tiles(KArgs a) {
  constexpr int kAT = AT;                            // accumulation tile (32 = the CCL tile width)
  constexpr int kARW = kAT + 4, kARH = kAT + 3;      // staged region incl. the halo
  constexpr int kARN = kARW * kARH;
  constexpr int kAPT = (kARN + 255) / 256;           // staged pixels per thread
  __shared__ TileAcc T;
  __shared__ int sfin[kARN];
  __shared__ uint8_t smask[kARN], scls[kARN];
  const int b = blockIdx.z;
  const int cw = a.cw, ch = a.ch, bins = a.bins;
  const int x0 = blockIdx.x * kAT, y0 = blockIdx.y * kAT;
  FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
  if (f.flag[1]) return;  // root pool exhausted: no records for this frame
  f.fb = f.flag[0];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < kTSlots; i += 256) {
    T.key[i] = 0; T.s00[i] = 0; T.s10[i] = 0; T.s01[i] = 0;
  }
  for (int i = tid; i < kTSlots * kDenseBins; i += 256) T.hist[i] = 0;
  const uint8_t* lab = a.labels + (size_t)b * a.H * a.W;
  {  // stage: all first-level loads, then all second-level (cidx) loads
    int lv[kAPT];
#pragma unroll
    for (int k = 0; k < kAPT; ++k) {
      const int i = tid + k * 256;
      const int gx = x0 - 2 + i % kARW, gy = y0 - 2 + i / kARW;
      const bool in = i < kARN && gx >= 0 && gx < cw && gy >= 0 && gy < ch;
      lv[k] = 0;
      if (in) {
        const int q = gy * cw + gx;
        lv[k] = f.L[q + 1];
        smask[i] = f.mask[q];
        int c = lab[gy * a.W + gx];
        scls[i] = (uint8_t)(c >= bins ? bins - 1 : c);
      } else if (i < kARN) {
        smask[i] = 0;
        scls[i] = 0;
      }
    }
#pragma unroll
    for (int k = 0; k < kAPT; ++k) {
      const int i = tid + k * 256;
      if (i < kARN) sfin[i] = lv[k] == 0 ? 0 : f.cidx[lv[k] - 1];
    }
  }
  __syncthreads();
  auto LI = [&](int gx, int gy) { return (gy - y0 + 2) * kARW + (gx - x0 + 2); };
  const int tx = tid % kAT, ty0 = tid / kAT;  // 256 / kAT rows per round
#pragma unroll 1
  for (int k = 0; k < kAT * kAT / 256; ++k) {
    const int x = x0 + tx, y = y0 + ty0 + (256 / kAT) * k;
    const bool own = x < cw && y < ch;
    // pieces in 32 bits: 6x + 3 < 2^19 for x < 65536
    int fnode = 0, f00 = 0, f10 = 0, f01 = 0;
    int bn[2] = {0, 0}, b00[2] = {0, 0}, b10[2] = {0, 0}, b01[2] = {0, 0};
    int np = 0, c = 0, rc[4] = {-1, -1, -1, -1};
    if (own) {
      const int i0 = LI(x, y);
      const bool m0 = smask[i0] != 0;
      const int n0 = sfin[i0];
      np = n0;
      c = scls[i0];
      if (x + 1 < cw && y + 1 < ch) {
        const int TX[4] = {1, 2, 1, 2}, TY[4] = {1, 1, 2, 2};
        const int node[4] = {n0, sfin[i0 + 1], sfin[i0 + kARW], sfin[i0 + kARW + 1]};
        const bool fg[4] = {m0, smask[i0 + 1] != 0, smask[i0 + kARW] != 0, smask[i0 + kARW + 1] != 0};
        int nf = 0, missing = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (fg[q]) { ++nf; fnode = node[q]; } else { missing = q; }
        }
        const int X = x, Y = y;
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
        for (int q = 0; q < 4; ++q) {
          if (fg[q] || node[q] == 0) continue;
          bool first = true;
          int cnt = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (!fg[j] && node[j] == node[q]) {
              ++cnt;
              if (j < q) first = false;
            }
          }
          if (!first) continue;
          if (nb < 2) {
            bn[nb] = node[q];
            if (cnt >= 2) { b00[nb] = 2; b10[nb] = 6 * X + 3; b01[nb] = 6 * Y + 3; }
            else { b00[nb] = 1; b10[nb] = 3 * X + TX[q]; b01[nb] = 3 * Y + TY[q]; }
            ++nb;
          }
        }
      }
      // hole rings, counted from the hole side exactly as in k_accum
      if (!m0 && np != 0 && !(a.dbg & 2)) {
        const int nx[4] = {x - 1, x + 1, x, x}, ny[4] = {y, y, y - 1, y + 1};
        const bool okn[4] = {x > 0, x + 1 < cw, y > 0, y + 1 < ch};
        bool fgn[4], any = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          fgn[q] = okn[q] && smask[LI(nx[q], ny[q])];
          any |= fgn[q];
        }
        if (any) {
          const int par = parent_of(f, cw, np);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (!fgn[q]) continue;
            const int rx = nx[q], ry = ny[q];
            int px[3] = {-1, -1, -1}, py[3] = {0, 0, 0};
            if (q == 0) {
              if (rx > 0) { px[0] = rx - 1; py[0] = ry; }
            } else if (q == 2) {
              if (rx > 0) { px[0] = rx - 1; py[0] = ry; }
              if (rx + 1 < cw) { px[1] = rx + 1; py[1] = ry; }
              if (ry > 0) { px[2] = rx; py[2] = ry - 1; }
            } else if (q == 3) {
              if (rx > 0) { px[0] = rx - 1; py[0] = ry; }
              if (rx + 1 < cw) { px[1] = rx + 1; py[1] = ry; }
            }
            const int ir = LI(rx, ry);
            bool first = true;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              if (px[j] < 0) continue;
              const int iq = LI(px[j], py[j]);
              if (!smask[iq] && sfin[iq] == np) first = false;
            }
            if (sfin[ir] != par || !first) continue;
            rc[q] = scls[ir];
          }
        }
      }
    }
    if (!(a.dbg & 8)) {
      tagg(T, f, cw, fnode, f00, f10, f01);
      tagg(T, f, cw, bn[0], b00[0], b10[0], b01[0]);
      tagg(T, f, cw, bn[1], b00[1], b10[1], b01[1]);
    }
    // class counts of the pixel's own component (and the rings of its hole contour)
    const int hn = (a.dbg & 1) ? 0 : np;
    const unsigned long long hact = __ballot(hn > 0);
    if (hact) {
      const int leader = __ffsll((long long)hact) - 1;
      const int lnp = __builtin_amdgcn_readlane(hn, leader);
      const bool uni = __all(hn <= 0 || hn == lnp);
      const int h = hn > 0 ? tslot(T, hn) : -1;  // one probe chain (uniform waves: same address)
      if (uni && h >= 0) {
        // node-uniform wave: one single-lane add per distinct class
        for (unsigned long long rem = hact; rem;) {
          const int l = __ffsll((long long)rem) - 1;
          const int cl = __builtin_amdgcn_readlane(c, l);
          const unsigned long long g = __ballot(hn > 0 && c == cl) & rem;
          if (lane == l) atomicAdd(&T.hist[h * kDenseBins + cl], __popcll(g));
          rem &= ~g;
        }
      } else if (hn > 0) {
        if (h >= 0) atomicAdd(&T.hist[h * kDenseBins + c], 1);
        else hist_global(f, cw, bins, hn, c, 1, false);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (hn > 0 && rc[q] >= 0) {
          if (h >= 0) atomicAdd(&T.hist[h * kDenseBins + rc[q]], 1 << 16);
          else hist_global(f, cw, bins, hn, rc[q], 1, true);
        }
      }
    }
  }
  __syncthreads();
  if (a.dbg & 16) return;
  // flush: each slot's ancestor chain once (one lane per slot), then fire-and-forget atomics
  if (tid < kTSlots) {
    const int node = T.key[tid];
    int d = 0, n = 0;
    if (node > 0 && !(a.dbg & 4)) {
      n = parent_of(f, cw, node);
      while (n != 0 && d < kAnc) {
        T.anc[tid][d++] = n;
        n = parent_of(f, cw, n);
      }
    }
    T.nanc[tid] = d;
    T.deep[tid] = n;  // != 0: the chain goes on past kAnc
  }
  __syncthreads();
  if (tid < kTSlots) {
    const int node = T.key[tid];
    if (node > 0 && T.s00[tid] != 0) {
      const int d00 = T.s00[tid];
      const unsigned long long d10 = T.s10[tid], d01 = T.s01[tid];  // (zero-extended)
      for (int k = -1; k < T.nanc[tid]; ++k) {
        const int n = k < 0 ? node : T.anc[tid][k];
        atomicAdd(f.t00 + n - 1, d00);
        atomicAdd(reinterpret_cast<unsigned long long*>(f.t10 + n - 1), d10);
        atomicAdd(reinterpret_cast<unsigned long long*>(f.t01 + n - 1), d01);
      }
      if (T.deep[tid] != 0) moments_up(f, cw, T.deep[tid], d00, (long long)d10, (long long)d01, 65536);
    }
  }
  for (int i = tid; i < kTSlots * kDenseBins; i += 256) {
    const int v = T.hist[i];
    if (v == 0) continue;
    const int sl = i / kDenseBins, cc = i - sl * kDenseBins;
    const int node = T.key[sl];
    const int own = v & 0xffff, ring = v >> 16;
    if (ring) atomicAdd(f.th + (size_t)(node - 1) * bins + cc, ring);
    if (own) {
      for (int k = -1; k < T.nanc[sl]; ++k)
        atomicAdd(f.th + (size_t)((k < 0 ? node : T.anc[sl][k]) - 1) * bins + cc, own);
      if (T.deep[sl] != 0) hist_global(f, cw, bins, T.deep[sl], cc, own, false);
    }
  }
}

// ---------------------------------------------------------------- select
// assign_frame (k_records, one workgroup per frame) hands the record slots to the first K passing
// contours in raster order of their discovery pixel: the passing roots of the root
// list are gathered in LDS and bitonic-sorted. The choice is deterministic (round 1
// took them in atomicAdd order, so with more than K passing contours the kept subset
// changed from run to run) and keeps the smallest discovery keys: among
// siblings those come LAST in findContours order, so they are the records the
// reference's LIFO buffer serves first (/root/reference/sem_seg_server.py:186-192,
// 52-60). Contours past K are counted in nslot[1]; the finalize phase flags the frame by a
// negative record count. Frames with more than kSortCap passing contours take a
// raster-order scan of every pixel instead. (Round 2 ran a full-frame k_select pass
// before this kernel: 20 us per 32 frames.)
__device__ __forceinline__ bool passes_n(const FrameWS& f, const KArgs& a, int n) {
  const int t = f.t00[n - 1];
  return t != 0 && (double)t * 0.5 >= a.min_area;
}

// label of pixel p if p is its component's root (first pixel) and the contour passes, else 0
__device__ __forceinline__ int passes_px(const FrameWS& f, const KArgs& a, int p) {
  const int n = fin(f, p);
  return n != 0 && f.rlist[n - 1] == p && passes_n(f, a, n) ? n : 0;
}

constexpr int kSortCap = 2048;  // (LDS: k_records shares CUs with the next step's model kernels)

// (record slots handed out here are also kept in LDS, s_sn / s_res, for the finalize
// phase of the same workgroup)
__device__ __forceinline__ void assign_frame(const KArgs& a, FrameWS& f, int* s_sn, int* s_res) {
  __shared__ int s_key[kSortCap];
  __shared__ int s_cnt, s_w[16];
  const int t = threadIdx.x;
  const int N = a.ch * a.cw;
  if (t == 0) s_cnt = 0;
  __syncthreads();
  const int nroot = f.nslot[3], base = f.flag[3];
  for (int i = t; i < nroot; i += 1024) {
    if (passes_n(f, a, base + i + 1)) {
      const int k = atomicAdd(&s_cnt, 1);
      if (k < kSortCap) s_key[k] = f.rlist[base + i];  // sorted by raster root
    }
  }
  __syncthreads();
  const int total = s_cnt;
  const int kept = min(total, a.K);
  if (total <= kSortCap) {
    int n2 = 1;
    while (n2 < total) n2 <<= 1;
    for (int i = total + t; i < n2; i += 1024) s_key[i] = 0x7fffffff;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = t; i < n2; i += 1024) {
          const int ij = i ^ j;
          if (ij > i) {
            const int u = s_key[i], v = s_key[ij];
            if ((u > v) == ((i & k) == 0)) { s_key[i] = v; s_key[ij] = u; }
          }
        }
        __syncthreads();
      }
    }
    for (int i = t; i < kept; i += 1024) {
      const int n = f.cidx[s_key[i]];  // a component root's cidx entry is its label
      f.slot_node[i] = n;
      s_sn[i] = n;
    }
  } else {
    const int wid = t >> 6, lane = t & 63;
    int base = 0;
    for (int c0 = 0; c0 < N && base < kept; c0 += 1024) {
      const int p = c0 + t;
      const int n = p < N ? passes_px(f, a, p) : 0;
      const bool ok = n != 0;
      const unsigned long long m = __ballot(ok);
      if (lane == 0) s_w[wid] = __popcll(m);
      __syncthreads();
      int wb = 0, tot = 0;
      for (int w = 0; w < 16; ++w) {
        wb += w < wid ? s_w[w] : 0;
        tot += s_w[w];
      }
      const int rank = base + wb + __popcll(m & ((1ull << lane) - 1));
      if (ok && rank < kept) {
        f.slot_node[rank] = n;
        s_sn[rank] = n;
      }
      base += tot;
      __syncthreads();
    }
  }
  if (t == 0) {
    f.nslot[0] = kept;
    f.nslot[1] = total - kept;
    s_res[0] = kept;
    s_res[1] = total - kept;
  }
  __syncthreads();
}

// ---------------------------------------------------------------- finalize
constexpr int kMaxDepth = 16;

__device__ __forceinline__ int disc_key(const FrameWS& f, int n) {
  const int r = f.rlist[n - 1];
  return f.mask[r] ? r : r - 1;
}

__device__ __forceinline__ int node_depth(const FrameWS& f, int cw, int n) {
  int d = 0;
  for (; n != 0; n = parent_of(f, cw, n)) ++d;
  return d;
}

// Does node a (depth da) come before node b (depth db) in findContours pre-order?
// (a is an ancestor of b, or at the first divergence a's branch has the larger key.)
__device__ bool precedes(const FrameWS& f, int cw, int a, int da, int b, int db) {
  int u = a, v = b;
  for (; db > da; --db) v = parent_of(f, cw, v);
  if (u == v) return true;   // a is an ancestor of b
  for (; da > db; --da) u = parent_of(f, cw, u);
  if (u == v) return false;  // b is an ancestor of a
  while (parent_of(f, cw, u) != parent_of(f, cw, v)) {
    u = parent_of(f, cw, u);
    v = parent_of(f, cw, v);
  }
  return disc_key(f, u) > disc_key(f, v);
}

__device__ __forceinline__ void finalize_frame(const KArgs& a, FrameWS& f, const int* s_sn, const int* s_res, int) {
  const int b = blockIdx.x, NT = blockDim.x;
  float* rec = a.records + (size_t)b * (1 + 5 * a.K);
  __shared__ int s_node[256];
  __shared__ int s_path[256][kMaxDepth];
  __shared__ int s_len[256];
  __shared__ int s_order[256];
  __shared__ int s_emit[256];
  __shared__ float s_val[256][5];
  __shared__ int s_deep;
  const int ns = min(s_res[0], min(a.K, 256));
  const int t = threadIdx.x;
  if (t == 0) s_deep = 0;
  __syncthreads();
  for (int i = t; i < ns; i += NT) {
    const int node = s_sn[i];
    s_node[i] = node;
    // ancestor chain (top first) of discovery keys
    int chain[kMaxDepth];
    int len = 0;
    for (int n = node; n != 0 && len < kMaxDepth; n = parent_of(f, a.cw, n)) chain[len++] = disc_key(f, n);
    for (int k = 0; k < len; ++k) s_path[i][k] = chain[len - 1 - k];
    s_len[i] = len;
    if (len == kMaxDepth) {
      // chain truncated (nesting deeper than kMaxDepth): order by parent walks instead
      int n = node, d = 0;
      for (; n != 0 && d <= kMaxDepth; n = parent_of(f, a.cw, n)) ++d;
      if (n != 0) s_deep = 1;
    }
    // statistics
    const int r = node - 1;
    const int* h = f.th + (size_t)r * a.bins;
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
  if (s_deep) {  // exact order at any depth: lift to equal depth, then walk to the LCA
    for (int i = t; i < ns; i += NT) {
      int rank = 0;
      const int di = node_depth(f, a.cw, s_node[i]);
      for (int j = 0; j < ns; ++j)
        if (j != i) rank += precedes(f, a.cw, s_node[j], node_depth(f, a.cw, s_node[j]), s_node[i], di);
      s_order[rank] = i;
    }
    __syncthreads();
  }
  for (int i = t; i < ns && !s_deep; i += NT) {
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
    rec[0] = s_res[1] > 0 ? -(float)n : (float)n;  // negative: contours dropped past K
  }
}

// Record slots and records in ONE workgroup per frame (round 2: k_select + k_assign +
// k_finalize, three launches): the slot assignment above, then the finalize phase.
__global__ __launch_bounds__(1024) void k_records(KArgs a) {
  __shared__ int s_sn[256], s_res[2];
  FrameWS f = frame_ws(a.ws, a.lay, a.B, blockIdx.x);
  if (f.flag[1]) {  // root pool exhausted (adversarial batch): flagged, no records
    if (threadIdx.x == 0) a.records[(size_t)blockIdx.x * (1 + 5 * a.K)] = __builtin_nanf("");
    return;
  }
  f.fb = f.flag[0];
  assign_frame(a, f, s_sn, s_res);
  finalize_frame(a, f, s_sn, s_res, 0);
}


#ifdef SSA_POST_DEBUG
__global__ void k_dbg_reset(KArgs a) {
  for (int b = threadIdx.x; b < a.B; b += 256) {
    FrameWS f = frame_ws(a.ws, a.lay, a.B, b);
    f.flag[2] = 0;
    f.flag[4] = 0;
  }
}
#endif

}  // namespace

size_t post_workspace_bytes(int B, int H, int W, int K, int num_bins) {
  return layout(B, H, W, K, num_bins).total(B);
}

void postprocess(const PostParams& p, hipStream_t s) {
  if (p.K > 256) throw std::invalid_argument("postprocess: K > 256");
  if (p.H > 65535 || p.W > 65535)  // k_accum's 32-bit wave sums of 6x + 3 pieces
    throw std::invalid_argument("postprocess: maps larger than 65535 pixels per side");
  if (((long long)layout(p.B, p.H, p.W, p.K, p.num_bins).P + 1) * p.num_bins * 2 >= (1ll << 31))  // histogram keys
    throw std::invalid_argument("postprocess: root pool * classes too large for 32-bit histogram keys");
  if (p.crop_h > p.H || p.crop_w > p.W || p.crop_h <= 0 || p.crop_w <= 0)
    throw std::invalid_argument("postprocess: bad crop");
  if (p.accum < 0 || p.accum > 2) throw std::invalid_argument("postprocess: accum 0 (strips), 1 (32^2 tiles), 2 (64^2)");
  const int accum = p.num_bins > kDenseBins ? 0 : p.accum;  // the tile tables count <= 32 classes
  KArgs a;
  a.labels = p.labels;
  a.B = p.B; a.H = p.H; a.W = p.W; a.ch = p.crop_h; a.cw = p.crop_w;
  a.thr = p.thr; a.K = p.K; a.bins = p.num_bins; a.min_area = p.min_area;
  a.ws = static_cast<char*>(p.ws);
  a.lay = layout(p.B, p.H, p.W, p.K, p.num_bins);
  a.records = p.records;
  a.dbg = 0;
#ifdef SSA_POST_DEBUG
  // ablation / staging knobs: debug builds only (-DSSA_POST_DEBUG), never in the
  // production launch path
  {
    const char* e = getenv("SSA_POST_DBG");
    a.dbg = e ? atoi(e) : 0;
  }
#endif
  // the per-frame counters are zeroed inside k_ccl_local (a kernel, not hipMemsetAsync:
  // a memset node captured by torch.cuda.graph faulted on its second replay on ROCm 7.x)
  const int N = p.crop_h * p.crop_w;
  const dim3 blk(256);
  const dim3 gp(cdiv(N, 256), p.B);
  // SSA_POST_STAGES=n (debug) launches only the first n stages
#ifdef SSA_POST_DEBUG
  const int stages = [] {  // read per call (host only; graph capture records one value)
    const char* e = getenv("SSA_POST_STAGES");
    return e ? atoi(e) : 99;
  }();
#else
  constexpr int stages = 99;
#endif
  int st = 0;
  const dim3 gt(cdiv(p.crop_w, TW), cdiv(p.crop_h, TH), p.B);
  if (st++ < stages) hipLaunchKernelGGL(k_ccl_local, gt, dim3(kCclThreads), 0, s, a, p.palette);
  {
    const int tx_n = cdiv(p.crop_w, TW), ty_n = cdiv(p.crop_h, TH);
    const int nt = tx_n * ty_n;
    const int lines = (ty_n - 1) + 2 + 2 * (tx_n - 1) + 2;
    if (st++ < stages)
      hipLaunchKernelGGL(k_ccl_edges, dim3(cdiv(std::max(p.crop_w, p.crop_h), kEdgeThreads), lines, p.B),
                         dim3(kEdgeThreads), 0, s, a);
    const size_t lds = (size_t)(2 * (kMergeCap + 1) + kMergeCap + nt + 1 + 1024 + 3) * 4;
    if (lds > 160 * 1024) throw std::invalid_argument("postprocess: crop too large for the LDS merge (> ~1800^2 pixels)");
    static bool attr = false;
    if (!attr) {
      check(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ccl_merge),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
            "k_ccl_merge attr");
      attr = true;
    }
    // B merge workgroups + the union-find frames' relabel workgroups (idle unless flagged)
    if (st++ < stages)
      hipLaunchKernelGGL(k_ccl_merge, dim3(p.B + std::min(kFbBlocks, cdiv(N, 1024))), dim3(1024), lds, s, a);
  }
  // strip-privatised pass: kQuadBlocks strips per frame (SSA_QUAD_BLOCKS overrides, tuning)
  // rounds of 256 pixels per block chosen first, so no block ends with a near-empty round
  // (771-pixel strips at 256 blocks per frame ran a 4th round for 3 pixels)
#ifdef SSA_POST_DEBUG
  const char* qb_env = getenv("SSA_QUAD_BLOCKS");
#else
  const char* qb_env = nullptr;
#endif
  // small batches get more, shorter strips so the grid still covers the 256 CUs (batch 1:
  // 772 one-round blocks instead of 193 four-round blocks)
  const int qtarget = qb_env ? std::max(1, atoi(qb_env)) : std::max(kQuadBlocks, 2048 / p.B);
  const int rounds = std::max(1, N / (256 * qtarget));
  const int qblocks = cdiv(N, 256 * rounds) * (256 / kAccThreads);
  if (st++ < stages) {
    if (accum == 1)
      hipLaunchKernelGGL(k_accum_tiles<32>, dim3(cdiv(p.crop_w, 32), cdiv(p.crop_h, 32), p.B), dim3(256), 0, s, a);
    else if (accum == 2)
      hipLaunchKernelGGL(k_accum_tiles<64>, dim3(cdiv(p.crop_w, 64), cdiv(p.crop_h, 64), p.B), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(k_accum, dim3(qblocks, p.B), dim3(kAccThreads), 0, s, a);
  }
  if (st++ < stages) hipLaunchKernelGGL(k_records, dim3(p.B), dim3(1024), 0, s, a);
#ifdef SSA_POST_DEBUG
  if (stages < 3) hipLaunchKernelGGL(k_dbg_reset, dim3(1), dim3(256), 0, s, a);  // k_ccl_merge's resets
#endif
  check_launch("postprocess");
}

}  // namespace ssa
