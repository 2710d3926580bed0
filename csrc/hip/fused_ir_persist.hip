// Persistent fused inverted residual for the high-resolution MobileNetV2 blocks
// (129^2 / 65^2 maps: blocks 1-6), gfx950.
//
//   out = project( relu6( dw3x3( relu6( expand(x) ) ) ) ) [+ x]
//
// Same math and LDS data flow as fused_ir.hip's tile kernel (input halo tile X in
// LDS; hidden channels streamed in 32-wide chunks: expand on MFMA -> fp16 chunk E
// in LDS -> packed-fp16 depthwise straight into the projection's MFMA B fragment ->
// fp16 MFMA projection into fp32 registers), re-organised around what the
// s_memtime timelines of that kernel showed: every workgroup re-fetched ALL block
// weights from L2 once per hidden chunk (expand, depthwise and projection slices:
// ~2.5k cycles of exposed latency per chunk), and paid a cold input-tile load per
// 55..121-pixel tile.
//
//   * persistent: a grid sized to the resident capacity walks the tiles; the whole
//     block's weights (<= ~64 KB for blocks 1-6) are staged into LDS ONCE per
//     workgroup, with +16-byte row padding so the per-lane fragment reads of the
//     expansion ([hid][Cin]) and projection ([Cout][hid]) weights are bank-conflict
//     free; per chunk, every weight operand is an LDS read;
//   * the next tile's input halo is prefetched into VGPRs while the current tile
//     computes and committed to LDS after its epilogue (the only global loads in
//     the steady state).
#include "common.h"
#include "kernels.h"

namespace ssa {

namespace {

typedef _Float16 f16;
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int kPNW = 4;      // waves per workgroup
constexpr int kPXPF = 8;     // max 16-byte input-tile loads per thread held for the prefetch
constexpr int kPMaxG = 4;    // max expansion pixel groups per wave (halo tile <= 256 pixels)

struct PIRArgs {
  const bf16* in; const bf16* we; const float* be; const f16* wd; const f16* bd;
  const f16* wp; const float* bp; bf16* out;
  int B, IH, IW, Cin, CinP, hidP, Cout, CoutP, OH, OW, stride, dil, residual, TY, TX, tiles_y,
      tiles_x, ntiles;
};

struct PLayout {  // byte offsets into dynamic LDS
  int we, wp, wd, bd, be, bp, X, E, total;
};

// Row pitch of the expanded chunk E, in 16-byte units (one halo pixel = 5 units:
// 32 fp16 channels + a 16-byte pad). A ds_read_b128 is serviced 16 lanes at a time,
// conflict-free when the 16 lanes hit 16 distinct 16-byte bank groups (mod 16).
// The depthwise reads 16 consecutive output pixels: within a row 5 * dx is distinct
// mod 16, and across the row wrap (lanes (r, x) and (r + 1, x'), x' - x in
// [-(TX - 1), 15 - TX]) the pitch RP must avoid RP + 5 (x' - x) == 0 mod 16, i.e.
// RP == 5 * TX mod 16 (stride 1). The unpadded pitch 5 * TIW put two lanes of every
// row-wrapping group on one bank group (2-way conflicts on every depthwise read).
__host__ __device__ inline int e_pitch(int TX, int TIW, int stride) {
  int rp = 5 * TIW;
  if (stride == 1)
    while ((rp - 5 * TX) % 16 != 0) ++rp;
  return rp;
}

__host__ __device__ inline PLayout playout(int CinP, int hidP, int CoutP, int in_groups, int e_bytes) {
  PLayout l;
  int o = 0;
  l.we = o; o += hidP * (CinP + 8) * 2;
  l.wp = o; o += CoutP * (hidP + 8) * 2;
  l.wd = o; o += 9 * hidP * 2;
  l.bd = o; o += hidP * 2;
  o = (o + 15) & ~15;
  l.be = o; o += hidP * 4;
  l.bp = o; o += CoutP * 4;
  o = (o + 15) & ~15;
  l.X = o; o += in_groups * 16 * (CinP + 8) * 2;
  l.E = o; o += e_bytes > in_groups * 16 * 40 * 2 ? e_bytes : in_groups * 16 * 40 * 2;
  l.total = o;
  return l;
}

template <int NSUB, int KS, int GPW, int NW>
__global__ __launch_bounds__(64 * NW) void fused_ir_persist_kernel(PIRArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int CinP = KS * 32;
  constexpr int XS = CinP + 8, ES = 40, WES = CinP + 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = a.stride, dl = a.dil;
  const int TIH = (a.TY - 1) * s + 2 * dl + 1, TIW = (a.TX - 1) * s + 2 * dl + 1;
  const int in_px = TIH * TIW;
  const int in_groups = (in_px + 15) / 16;
  const int hidP = a.hidP, WPS = hidP + 8;
  const int RPE = e_pitch(a.TX, TIW, s) * 8;  // E row pitch in fp16 elements
  const PLayout L = playout(CinP, hidP, a.CoutP, in_groups, TIH * RPE * 2 + 256);
  bf16* sWe = reinterpret_cast<bf16*>(smem + L.we);
  f16* sWp = reinterpret_cast<f16*>(smem + L.wp);
  f16* sWd = reinterpret_cast<f16*>(smem + L.wd);
  f16* sBd = reinterpret_cast<f16*>(smem + L.bd);
  float* sBe = reinterpret_cast<float*>(smem + L.be);
  float* sBp = reinterpret_cast<float*>(smem + L.bp);
  bf16* X = reinterpret_cast<bf16*>(smem + L.X);
  f16* E = reinterpret_cast<f16*>(smem + L.E);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;

  // ---- stage the block's weights once (16-byte copies into padded rows)
  for (int i = tid; i < hidP * (CinP / 8); i += NT) {
    const int r = i / (CinP / 8), c = (i % (CinP / 8)) * 8;
    st8(sWe + r * WES + c, ld8(a.we + (size_t)r * CinP + c));
  }
  for (int i = tid; i < a.CoutP * (hidP / 8); i += NT) {
    const int r = i / (hidP / 8), c = (i % (hidP / 8)) * 8;
    *reinterpret_cast<f16x8*>(sWp + r * WPS + c) = *reinterpret_cast<const f16x8*>(a.wp + (size_t)r * hidP + c);
  }
  for (int i = tid; i < 9 * hidP / 8; i += NT)
    *reinterpret_cast<f16x8*>(sWd + i * 8) = *reinterpret_cast<const f16x8*>(a.wd + i * 8);
  for (int i = tid; i < hidP / 8; i += NT)
    *reinterpret_cast<f16x8*>(sBd + i * 8) = *reinterpret_cast<const f16x8*>(a.bd + i * 8);
  for (int i = tid; i < hidP; i += NT) sBe[i] = a.be[i];
  for (int i = tid; i < a.CoutP; i += NT) sBp[i] = a.bp[i];

  // ---- input halo tile: global -> registers (prefetch) -> LDS
  constexpr int cpp = CinP / 8;  // 16-byte pieces per pixel
  const int xpieces = in_groups * 16 * cpp;
  const int ntile_img = a.tiles_y * a.tiles_x;
  bf16x8 xr[kPXPF];
  auto load_x = [&](int tile) {
    const int b = tile / ntile_img, t = tile - b * ntile_img;
    const int iy0 = (t / a.tiles_x) * a.TY * s - dl, ix0 = (t % a.tiles_x) * a.TX * s - dl;
#pragma unroll
    for (int q = 0; q < kPXPF; ++q) {
      const int i = tid + q * NT;
      bf16x8 v = zero8();
      if (i < xpieces) {
        const int ip = i / cpp, c = (i % cpp) * 8;
        const int ty = ip / TIW, tx = ip - ty * TIW;
        const int iy = iy0 + ty, ix = ix0 + tx;
        if (ip < in_px && c < a.Cin && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW)
          v = ld8(a.in + (((size_t)b * a.IH + iy) * a.IW + ix) * a.Cin + c);
      }
      xr[q] = v;
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int q = 0; q < kPXPF; ++q) {
      const int i = tid + q * NT;
      if (i < xpieces) st8(X + (size_t)(i / cpp) * XS + (i % cpp) * 8, xr[q]);
    }
  };

  int tile = blockIdx.x;
  if (tile < a.ntiles) load_x(tile);
  store_x();
  __syncthreads();

  // Tile-invariant per-lane geometry, computed once (the PMC profile of the first
  // version showed ~38 VALU instructions per MFMA, mostly the integer divisions
  // and address math of the halo pixels redone for every tile and every chunk):
  //  * expansion groups of this wave: halo pixel (ty, tx), X / E element offsets;
  //  * output groups: tile-local (py, px) and the depthwise base offset in E.
  constexpr int MAXG = kPMaxG;  // expansion groups per wave
  int gip[MAXG], gyx[MAXG];    // halo pixel index; (ty << 16 | tx), ty = 0x7fff for padding lanes
#pragma unroll
  for (int k = 0; k < MAXG; ++k) {
    const int ip = (wid + k * NW) * 16 + r16;
    const int ty = ip / TIW;
    gip[k] = ip;
    gyx[k] = ((ip < in_px ? ty : 0x7fff) << 16) | (ip - ty * TIW);
  }
  const int ngroups_w = (in_groups - wid + NW - 1) / NW;  // expansion groups this wave owns
  int pofs[GPW], opy[GPW], opx[GPW];
  bool pin[GPW];
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    const int p = (wid * GPW + g) * 16 + r16;
    opy[g] = p / a.TX;
    opx[g] = p - opy[g] * a.TX;
    pin[g] = p < a.TY * a.TX;
    pofs[g] = pin[g] ? opy[g] * s * RPE + opx[g] * s * ES : 0;
  }
  const int dw_row = dl * RPE, dw_col = dl * ES;  // tap strides in E (elements)
  int geo[MAXG];  // E element offset of each expansion group's halo pixel
#pragma unroll
  for (int k = 0; k < MAXG; ++k) {
    const int ty = gyx[k] >> 16, tx = gyx[k] & 0xffff;
    geo[k] = ty < 0x7fff ? ty * RPE + tx * ES : TIH * RPE;  // padding lanes: scratch slack past E
  }

  const f16x8 h0 = {0, 0, 0, 0, 0, 0, 0, 0}, h6 = {6, 6, 6, 6, 6, 6, 6, 6};
  for (; tile < a.ntiles; tile += gridDim.x) {
    const int b = tile / ntile_img, t = tile - b * ntile_img;
    const int oy0 = (t / a.tiles_x) * a.TY, ox0 = (t % a.tiles_x) * a.TX;
    const int iy0 = oy0 * s - dl, ix0 = ox0 * s - dl;
    const int next = tile + gridDim.x;
    if (next < a.ntiles) load_x(next);  // in flight under this tile's chunks

    // this tile's image-border masks
    unsigned inside = 0;
#pragma unroll
    for (int k = 0; k < MAXG; ++k)
      if ((unsigned)(iy0 + (gyx[k] >> 16)) < (unsigned)a.IH && (unsigned)(ix0 + (gyx[k] & 0xffff)) < (unsigned)a.IW)
        inside |= 1u << k;
    bool pval[GPW];
#pragma unroll
    for (int g = 0; g < GPW; ++g) pval[g] = pin[g] && oy0 + opy[g] < a.OH && ox0 + opx[g] < a.OW;
    f32x4 acc[GPW][NSUB];
#pragma unroll
    for (int g = 0; g < GPW; ++g)
#pragma unroll
      for (int n = 0; n < NSUB; ++n) acc[g][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int c0 = 0; c0 < hidP; c0 += 32) {
      // ---- expand this chunk over the halo tile -> E (fp16, relu6, zero outside)
      bf16x8 wfr[2][KS];
      f32x4 bias[2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
        for (int k = 0; k < KS; ++k) wfr[sub][k] = ld8(sWe + (c0 + sub * 16 + r16) * WES + k * 32 + kq * 8);
        bias[sub] = *reinterpret_cast<const f32x4*>(sBe + c0 + sub * 16 + kq * 4);
      }
#pragma unroll
      for (int kg = 0; kg < MAXG; ++kg) {
        if (kg >= ngroups_w) break;
        bf16x8 xf[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k) xf[k] = ld8(X + gip[kg] * XS + k * 32 + kq * 8);
        const bool in_img = (inside >> kg) & 1u;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          f32x4 e = bias[sub];
#pragma unroll
          for (int k = 0; k < KS; ++k) e = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[sub][k], xf[k], e, 0, 0, 0);
          f16x4 o = {(f16)e[0], (f16)e[1], (f16)e[2], (f16)e[3]};
          o = __builtin_elementwise_min(__builtin_elementwise_max(o, h0.lo), h6.lo);
          if (!in_img) o = h0.lo;  // zero padding applies to the expanded tensor
          *reinterpret_cast<f16x4*>(E + geo[kg] + sub * 16 + kq * 4) = o;
        }
      }
      __syncthreads();

      // ---- depthwise (packed fp16): lane -> 8 channels (kq*8..) of its pixel per group
      f16x8 wdv[9];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) wdv[tap] = *reinterpret_cast<const f16x8*>(sWd + tap * hidP + c0 + kq * 8);
      const f16x8 bdv = *reinterpret_cast<const f16x8*>(sBd + c0 + kq * 8);
      f16x8 af[NSUB];
#pragma unroll
      for (int n = 0; n < NSUB; ++n)
        af[n] = *reinterpret_cast<const f16x8*>(sWp + (n * 16 + r16) * WPS + c0 + kq * 8);
      f16x8 d[GPW];
#pragma unroll
      for (int g = 0; g < GPW; ++g) {
        f16x8 v[9];
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
          v[tap] = *reinterpret_cast<const f16x8*>(E + pofs[g] + (tap / 3) * dw_row + (tap % 3) * dw_col + kq * 8);
        d[g] = bdv;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) d[g] = v[tap] * wdv[tap] + d[g];
        d[g] = __builtin_elementwise_min(__builtin_elementwise_max(d[g], h0), h6);
      }
      // ---- project chunk (fp16 MFMA, fp32 accumulate)
#pragma unroll
      for (int n = 0; n < NSUB; ++n)
#pragma unroll
        for (int g = 0; g < GPW; ++g)
          acc[g][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[n], d[g], acc[g][n], 0, 0, 0);
      __syncthreads();  // E is rewritten by the next chunk
    }

    // ---- epilogue: + bias (+ residual from the LDS input tile), bf16 store
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      if (!pval[g]) continue;
      bf16* op = a.out + (((size_t)b * a.OH + oy0 + opy[g]) * a.OW + ox0 + opx[g]) * a.Cout;
      const bf16* rp = X + (size_t)((opy[g] * s + dl) * TIW + opx[g] * s + dl) * XS;
#pragma unroll
      for (int n = 0; n < NSUB; ++n) {
        const int co = n * 16 + kq * 4;
        if (co >= a.Cout) continue;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = acc[g][n][q] + sBp[co + q];
          if (a.residual) v[q] += (float)rp[co + q];
        }
        if (co + 3 < a.Cout) {
          bf16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = (bf16)v[q];
          *reinterpret_cast<bf16x4*>(op + co) = o;
        } else {
          for (int q = 0; q < 4; ++q)
            if (co + q < a.Cout) op[co + q] = (bf16)v[q];
        }
      }
    }
    // ---- commit the prefetched next input tile (everyone is done with X)
    __syncthreads();
    if (next < a.ntiles) store_x();
    __syncthreads();
  }
}

template <int NSUB, int KS, int GPW, int NW>
void launch_persist(const PIRArgs& a, size_t lds, hipStream_t st) {
  static int ncu = 0;
  if (ncu == 0) {
    check(hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_ir_persist_kernel<NSUB, KS, GPW, NW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
          "fused_ir_persist attr");
    int dev = 0;
    check(hipGetDevice(&dev), "hipGetDevice");
    check(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev), "cu count");
  }
  // resident capacity for THIS launch's LDS size (occupancy query per call is cheap
  // host work and keeps graph capture valid: nothing here touches the stream)
  int occ = 0;
  check(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &occ, reinterpret_cast<const void*>(&fused_ir_persist_kernel<NSUB, KS, GPW, NW>), 64 * NW, lds),
        "occupancy");
  occ = occ < 1 ? 1 : occ;
  const int grid = std::min(a.ntiles, ncu * occ);
  hipLaunchKernelGGL((fused_ir_persist_kernel<NSUB, KS, GPW, NW>), dim3(grid), dim3(64 * NW), lds, st, a);
  check_launch("fused_ir_persist");
}

}  // namespace

size_t fused_ir_persist_lds(int CinP, int hidP, int Cout, int stride, int dil, int TY, int TX, int nw) {
  if (nw != 4 && nw != 8) return 0;
  const int TIH = (TY - 1) * stride + 2 * dil + 1, TIW = (TX - 1) * stride + 2 * dil + 1;
  const int in_groups = (TIH * TIW + 15) / 16;
  const int CoutP = (Cout + 15) / 16 * 16;
  if ((size_t)in_groups * 16 * (CinP / 8) > (size_t)kPXPF * 64 * nw) return 0;  // prefetch registers
  if (in_groups > kPMaxG * nw) return 0;                                       // expansion groups per wave
  if ((TY * TX + 15) / 16 > 2 * nw) return 0;                                  // output groups per wave
  const int RPE = e_pitch(TX, TIW, stride) * 8;
  return (size_t)playout(CinP, hidP, CoutP, in_groups, TIH * RPE * 2 + 256).total;
}

void fused_ir_persist(const FusedIRParams& p, hipStream_t st) {
  if (!p.we || !p.wd_h || !p.bd_h || !p.wp_h) throw std::invalid_argument("fused_ir_persist: needs expansion + fp16 weights");
  if (p.dil < 1 || p.TX < 1 || p.TY < 1) throw std::invalid_argument("fused_ir_persist: bad tile");
  if (p.Cin % 8 || p.hidP % 32 || p.CinP % 32 || p.CinP < p.Cin)
    throw std::invalid_argument("fused_ir_persist: bad channel padding");
  if (p.residual && (p.stride != 1 || p.Cin != p.Cout)) throw std::invalid_argument("fused_ir_persist: bad residual");
  const int nw = p.nw == 8 ? 8 : 4;
  const int groups = (p.TY * p.TX + 15) / 16;
  const int gpw = (groups + nw - 1) / nw;
  const size_t lds = fused_ir_persist_lds(p.CinP, p.hidP, p.Cout, p.stride, p.dil, p.TY, p.TX, nw);
  if (gpw > 2 || lds == 0 || lds > 160 * 1024) throw std::invalid_argument("fused_ir_persist: tile / weights too large");
  const int ty_n = cdiv(p.OH, p.TY), tx_n = cdiv(p.OW, p.TX);
  PIRArgs a{p.in, p.we, p.be, reinterpret_cast<const f16*>(p.wd_h), reinterpret_cast<const f16*>(p.bd_h),
            reinterpret_cast<const f16*>(p.wp_h), p.bp, p.out, p.B, p.IH, p.IW, p.Cin, p.CinP, p.hidP,
            p.Cout, (p.Cout + 15) / 16 * 16, p.OH, p.OW, p.stride, p.dil, p.residual, p.TY, p.TX, ty_n,
            tx_n, p.B * ty_n * tx_n};
  const int nsub = (p.Cout + 15) / 16, ks = p.CinP / 32;
#define PIR(N, K)                                                                          \
  if (nsub == N && ks == K) {                                                              \
    if (nw == 8) {                                                                         \
      if (gpw <= 1) launch_persist<N, K, 1, 8>(a, lds, st); else launch_persist<N, K, 2, 8>(a, lds, st); \
    } else {                                                                               \
      if (gpw <= 1) launch_persist<N, K, 1, 4>(a, lds, st); else launch_persist<N, K, 2, 4>(a, lds, st); \
    }                                                                                      \
    return;                                                                                \
  }
  PIR(2, 1) PIR(4, 1) PIR(4, 2) PIR(6, 2)
#undef PIR
  throw std::invalid_argument("fused_ir_persist: unsupported (Cout, Cin) combination");
}

}  // namespace ssa
