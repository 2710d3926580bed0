// Host launch interfaces of the gfx950 kernels. Every launcher takes raw device
// pointers plus the caller's stream, performs no allocation and no host sync, and
// is therefore capturable into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace ssa {

struct ConvParams {
  const bf16* in = nullptr;      // [B, IH, IW, Cin] NHWC
  const bf16* w = nullptr;       // [Cout, KH, KW, Cin]
  const float* bias = nullptr;   // [Cout]
  const float* img_bias = nullptr;  // optional [B, Cout], added per image
  const bf16* res = nullptr;     // optional residual [B, OH, OW, ldr]
  bf16* out = nullptr;           // [B, OH, OW, ldo], written at channel offset co_off
  int B = 0, IH = 0, IW = 0, Cin = 0, OH = 0, OW = 0, Cout = 0;
  int KH = 1, KW = 1, stride = 1, dil = 1;
  int ldo = 0, co_off = 0, ldr = 0, act = 0;
  int variant = 0;  // 0 auto, 1 direct, 2 LDS-staged, 3/4 LDS-DMA 3/2-stage, 5/6 LDS-DMA 128x256/256x256
  // optional GEMM-row -> output-pixel permutation (-1 = padding row) of Mp rows;
  // LDS-DMA variants only (tap-validity-grouped tiles for dilated convs)
  const int* perm = nullptr;
  int Mp = 0;
};
void conv_gemm(const ConvParams& p, hipStream_t s);
// n (<= 4) independent LDS-DMA convs with one Cout in one grid; order[i] =
// (group << 24) | tile picks block i's tile (row-major (m-tile, n-tile) of that
// conv's GEMM, BM x BN of the variant: 5 128x256, 6 256x256, 8 128x256 3-stage,
// 10 128x128 4-stage, 11 128x128 2-stage).
void conv_gemm_grouped(const ConvParams* ps, int n, const int* order, int nblocks, int variant,
                       hipStream_t s, int ks = 1, float* part = nullptr, int* cnt = nullptr,
                       int cnt_stride = 0);

// Pointwise conv, weight-streamed (pw_conv.hip). w is host-packed per 64-channel
// chunk: weights in MFMA fragment order [4][ceil(K/32)][64 lanes][8] bf16 followed by
// 1 KiB holding the chunk's 64 fp32 biases, zero-padded (hip_ops.pack_pw_weights).
struct PwConvParams {
  const bf16* in = nullptr;        // [M, K]
  const bf16* w = nullptr;         // packed weights + biases
  const float* img_bias = nullptr; // optional [M / HW, N]
  const bf16* res = nullptr;       // optional [M, ldr]
  bf16* out = nullptr;             // [M, ldo] at channel offset co_off
  int M = 0, K = 0, N = 0, HW = 1, ldo = 0, co_off = 0, ldr = 0, act = 0;
  int mt = 2;   // 16*mt pixels per wave (2 or 4)
  int nch = 1;  // 64-channel chunks per workgroup
  int out_f16 = 0;  // 1: write fp16 instead of bf16 (same 2-byte layout)
};
void pw_conv(const PwConvParams& p, hipStream_t s);

// Dilated KxK stride-1 conv as a tap loop of weight-streamed MFMA GEMMs
// (tap_conv.hip; the ASPP atrous branches). w is host-packed (hip_ops.pack_tap_weights):
// [tap][ceil(Cout/128)][8 subtiles][ceil(Cin/32)][64 lanes][8] bf16, zero-padded.
struct TapConvParams {
  const bf16* in = nullptr;     // [B, H, W, Cin]
  const bf16* w = nullptr;      // packed
  const float* bias = nullptr;  // [ceil(Cout/128)*128] (zero-padded)
  bf16* out = nullptr;          // [B, H, W, ldo] at channel offset co_off
  const int* perm = nullptr;    // optional row -> pixel permutation (tap_group_perm), Mp rows
  int Mp = 0;
  int B = 0, H = 0, W = 0, Cin = 0, Cout = 0, KH = 3, KW = 3, dil = 1, ldo = 0, co_off = 0, act = 0;
};
void tap_conv(const TapConvParams& p, hipStream_t s);
int tap_conv_group_channels();  // output channels per workgroup (packing granule)
int pw_conv_supported_ks(int K);  // 0 if K has no instantiation

// int8 implicit-GEMM conv (int8 MFMA, int32 accumulate). scale[n] = in_scale *
// w_scale[n]; out_mode 0 -> int8 out (round(v * inv_out_scale), clamp +-127),
// 1 -> bf16 out. res (optional) is int8 [M, Cout] with res_scale.
struct ConvI8Params {
  const int8_t* in = nullptr;   // [B, IH, IW, Cin]
  const int8_t* w = nullptr;    // [Cout, KH, KW, Cin]
  const float* scale = nullptr; // [Cout]
  const float* bias = nullptr;  // [Cout]
  const float* img_bias = nullptr;
  const int8_t* res = nullptr;
  float res_scale = 0.f;
  void* out = nullptr;
  float inv_out_scale = 1.f;
  int out_mode = 0;
  int B = 0, IH = 0, IW = 0, Cin = 0, OH = 0, OW = 0, Cout = 0;
  int KH = 1, KW = 1, stride = 1, dil = 1, ldo = 0, co_off = 0, act = 0;
  int variant = 0;  // 0 auto, 1 register-fed, 2/3/4/7/8 LDS-DMA 128x128 / 128x256 / 256x128 / 160x128 / 96x128
  const int* perm = nullptr;  // LDS-DMA variants: GEMM row -> output pixel (-1 = padding row), Mp rows
  int Mp = 0;
};
void conv_i8(const ConvI8Params& p, hipStream_t s);
// Up to 4 independent int8 convs (the ASPP branches: one input, disjoint channel slices of
// the concat buffer) in ONE LDS-DMA grid: block i runs tile order[i] = (group << 24) | tile
// (host-sorted by live-tap work, heaviest first). variant: 2/3/4/7/8 (the tile shape).
void conv_i8_grouped(const ConvI8Params* ps, int n, const int* order, int nblocks, int variant,
                     hipStream_t s);
void maxpool3x3s2_i8(const int8_t* in, int8_t* out, int B, int IH, int IW, int C, int OH, int OW,
                     hipStream_t s);
// int8 GAP -> fp32 mean * scale; ws: B * 16 * C floats
void global_avgpool_i8(const int8_t* in, float* out, float* ws, int B, int HW, int C, float scale,
                       hipStream_t s);

// Fused MobileNetV2 inverted residual (expand 1x1 + ReLU6 -> dw 3x3 + ReLU6 ->
// project 1x1 [+ residual]), dilation 1. Weights are host-padded: CinP, hidP
// multiples of 32 (CinP <= 64), CoutP = 16 * ceil(Cout / 16).
struct FusedIRParams {
  const bf16* in = nullptr;   // [B, IH, IW, Cin]
  const bf16* we = nullptr;   // [hidP, CinP] or null (no expansion: hidP == CinP)
  const float* be = nullptr;  // [hidP]
  const float* wd = nullptr;  // [9, hidP]
  const float* bd = nullptr;  // [hidP]
  const bf16* wp = nullptr;   // [CoutP, hidP]
  const float* bp = nullptr;  // [CoutP]
  bf16* out = nullptr;        // [B, OH, OW, Cout]
  int B = 0, IH = 0, IW = 0, Cin = 0, CinP = 0, hidP = 0, Cout = 0, OH = 0, OW = 0;
  int stride = 1, residual = 0;
  int dil = 1;         // tile kernel only
  int TY = 0, TX = 0;  // > 0: general 2-D tile kernel (any dilation, CinP <= 160, CoutP <= 320)
  // tile kernel: fp16 copies of the depthwise weights [9, hidP], bias [hidP] and
  // projection weights [CoutP, hidP]
  const void* wd_h = nullptr;
  const void* bd_h = nullptr;
  const void* wp_h = nullptr;
  long long* trace = nullptr;  // debug timeline (128 slots), tile kernel only
};
void fused_inverted_residual(const FusedIRParams& p, hipStream_t s);
// Fused inverted residual over raster spans of the 33x33 maps (fused_ir_stream.hip):
// stride 1, dilation 1-2, Cin % 32 == 0, Cout % 16 == 0. w: host-packed chunk images
// (ops/fused_span.pack_fused_span, ReLU6 folded as a [0, 1] clamp: expansion / 6, depthwise
// bias / 6, projection x 6), table: span/halo table (fused_span.span_table) of S spans,
// hstride ints each.
struct FusedSpanParams {
  const bf16* in = nullptr;   // [B, H, W, Cin]
  const void* w = nullptr;    // [hidP / 32][(2*Cin/32 + Cout/16 + 1) KiB]
  const float* bp = nullptr;  // [Cout]
  const int* table = nullptr;
  bf16* out = nullptr;        // [B, H, W, Cout]
  int B = 0, H = 0, W = 0, Cin = 0, hidP = 0, Cout = 0, dil = 1, residual = 0;
  int S = 8, WR = 0, WCP = 0, hstride = 0;
  int npi = 0;                // fused_ir_stream variant (wave roles / ring slots)
  long long* trace = nullptr; // debug s_memtime timeline [B*S][2][64]
  int nh_max = 0;             // largest halo of the table (fused_ir_stream: <= 320)
  int hsplit = 1;             // fused_ir_stream: workgroups per span over the hidden chunks
  float* part = nullptr;      // hsplit > 1: fp32 partials [hsplit][B*H*W][Cout]
  int* cnt = nullptr;         // hsplit > 1: per-span tickets [B*S] for the in-launch combine (null:
                              // the caller runs stream_combine)
};
// Wave-specialised: expansion waves 0-3, depthwise+projection waves 4-7, LDS-DMA chunk ring.
void fused_ir_stream(const FusedSpanParams& p, hipStream_t s);
size_t fused_ir_stream_lds(int Cin, int Cout, int WR, int WCP, int nsl = 0);
// sum of the hidden-split partials + bias (+ residual) -> bf16 [M, Cout]
void stream_combine(const float* part, const float* bp, const bf16* res, bf16* out, int HS, long long M, int Cout,
                    hipStream_t st, int act = 0);
// Row-streaming fused inverted residual (fused_ir_band.hip): blocks with Cin <= 32,
// stride 1/2, dilation 1. blob: host-packed weights (hip_ops.pack_fused_band) with the
// section offsets below; R output rows per band, nslot E row buffers (1 or 2).
struct FusedBandParams {
  const bf16* in = nullptr;   // [B, IH, IW, Cin]
  const void* blob = nullptr;
  bf16* out = nullptr;        // [B, OH, OW, Cout]
  int B = 0, IH = 0, IW = 0, Cin = 0, OH = 0, OW = 0, Cout = 0, hidP = 0, stride = 1, residual = 0;
  int R = 8, nslot = 2, blob_bytes = 0, o_be = 0, o_wd = 0, o_bd = 0, o_wp = 0, o_bp = 0;
  int hs = 1;                 // 2: two waves per column group, each half the hidden channels
  int split = 1;              // 2: two column bands across the map width
};
void fused_ir_band(const FusedBandParams& p, hipStream_t s);
size_t fused_ir_band_lds(int stride, int hidP, int OW, int blob_bytes, int nslot, int hs = 1, int Cout = 0,
                         int split = 1);
int fused_ir_band_cols(int stride);
// Hidden-sliced variant (fused_ir_slice.hip): waves = nw column groups x hidP/32 hidden
// chunks, each wave's chunk weights in VGPRs; same blob as fused_ir_band (hs / split /
// nslot / blob_bytes unused).
// one_barrier: one workgroup barrier per input row (double-buffered E / D rows), else two
void fused_ir_slice(const FusedBandParams& p, int nw, hipStream_t s, bool one_barrier = false);
size_t fused_ir_slice_lds(int stride, int hidP, int OW, int Cout, int nw, bool one_barrier = false);
// Fused stem (3x3 s2, 3 -> 32, relu6, letterbox gather) + MobileNetV2 block 0
// (dw 3x3 on 32 ch + relu6, project 32 -> 16); weights: ws [32][32] bf16 with
// K = (ky*3+kx)*3 + c (RGB), bs [32] f32, wd [9][32] f16, bd [32] f16, wp [16][32] f16, bp [16].
struct StemBlock0Params {
  const uint8_t* frames = nullptr; const int32_t* lut_x = nullptr; const int32_t* lut_y = nullptr;
  const bf16* ws = nullptr; const float* bs = nullptr;
  const void* wd = nullptr; const void* bd = nullptr; const void* wp = nullptr;
  const float* bp = nullptr; bf16* out = nullptr;
  int B = 0, Hc = 0, Wc = 0, H = 0, W = 0, SH = 0, SW = 0, Cout = 16, TY = 8, TX = 16;
};
void stem_block0(const StemBlock0Params& p, hipStream_t s);
// Row-streaming stem + block 0 (stem_band.hip): bands of p.TY output rows x ceil(SW / nbx)
// columns; same weights as stem_block0 (p.TX unused).
// one_barrier: one workgroup barrier per stem row (double-buffered stem row), else two
void stem_band(const StemBlock0Params& p, int nbx, hipStream_t s, bool one_barrier = true);
size_t stem_band_lds(int SW, int nbx, int R);
// LDS bytes the tile kernel needs for a (TY, TX) tile (0 if the shape is unsupported).
size_t fused_ir_tile_lds(int CinP, int stride, int dil, int TY, int TX, int expand);

// DeepLabv3 head (aspp_head.hip): ASPP projection [M, K] x [K, 256] + bias + per-image
// bias + ReLU, then the logits 1x1 conv (256 -> ncls <= 32) from the on-chip projection
// tile. wp: [16 subtiles][K/32][64 lanes][8] bf16 (MFMA fragment order), wl: [2][8][64][8]
// bf16 (classes zero-padded to 32), bl: [32] fp32 (zero-padded).
struct AsppHeadParams {
  const bf16* cat = nullptr;        // [M, K] concatenated ASPP branches
  const bf16* wp = nullptr;
  const float* bp = nullptr;        // [256]
  const float* img_bias = nullptr;  // optional [M / HW, 256]
  const bf16* wl = nullptr;
  const float* bl = nullptr;
  bf16* out = nullptr;              // [M, ldo] logits (channels >= ncls written as 0 up to ldo)
  int M = 0, K = 0, N = 256, HW = 0, ncls = 0, ldo = 0;
  int G = 9;                        // 16-pixel groups per workgroup (1, 2, 3, 5, 9)
  int waves = 8;                    // 8 (2 projection subtiles per wave) or 16 (1)
};
void aspp_head(const AsppHeadParams& p, hipStream_t s);
size_t aspp_head_lds(int G, int K);

// Depthwise 3x3 (+bias, ReLU6) fused with the 1x1 projection (+bias [+ residual]):
// the depthwise output stays in registers as the projection's MFMA operand.
// Weights: wd [9, hid] fp32, wp [CoutP, hid] bf16 (CoutP = 16 * ceil(Cout / 16)).
struct DwProjectParams {
  const bf16* hid_in = nullptr;  // [B, IH, IW, hid]
  const float* wd = nullptr;
  const float* bd = nullptr;
  const bf16* wp = nullptr;
  const float* bp = nullptr;
  const bf16* res = nullptr;     // optional [B, OH, OW, Cout]
  bf16* out = nullptr;           // [B, OH, OW, Cout]
  int B = 0, IH = 0, IW = 0, hid = 0, Cout = 0, OH = 0, OW = 0, stride = 1, dil = 1;
};
void dw_project(const DwProjectParams& p, hipStream_t s);

// Depthwise + projection, weight-streamed (dw_proj.hip), fp16 internals. w is
// host-packed per 32-channel hidden chunk: [Cout/16 subtiles][64 lanes][8] fp16
// projection fragments, then [9][32] fp16 depthwise weights and [32] fp16 biases,
// padded to (Cout/16 + 1) KiB (hip_ops.pack_dw_proj).
struct DwProjFusedParams {
  const void* h = nullptr;     // [B, IH, IW, hid] expanded activations, fp16
  const void* w = nullptr;     // packed
  const float* bp = nullptr;   // [Cout] projection bias
  const bf16* res = nullptr;   // optional [B, OH, OW, Cout]
  bf16* out = nullptr;         // [B, OH, OW, Cout]
  int B = 0, IH = 0, IW = 0, hid = 0, Cout = 0, OH = 0, OW = 0, stride = 1, dil = 1;
  int waves = 4;               // 4 or 8 waves (16 pixels each) per workgroup
  int rows = 0;                // > 0: row-tile variant, this many output rows per workgroup
};
void dw_proj_fused(const DwProjFusedParams& p, hipStream_t s);

// Depthwise KxK (K=3) conv, NHWC, pad = dil, bias + act. w: [9, C] fp32.
void depthwise3x3(const bf16* in, const float* w, const float* bias, bf16* out, int B, int IH,
                  int IW, int C, int OH, int OW, int stride, int dil, int act, hipStream_t s);

// Fused letterbox preprocess + stem conv: uint8 BGR frames [B, Hc, Wc, 3] ->
// model pixel (y, x) = frame[lut_y[y], lut_x[x]] (or 0 where a lut is -1), RGB,
// x/127.5 - 1 -> KxK stride-s conv (pad K/2) 3 -> Cout, bias + act, NHWC bf16.
// w: [K*K*3, Cout] fp32 (tap-major, then input channel).
// out_inv_scale > 0: int8 output round(v * out_inv_scale) (int8 pipelines).
// Stem conv on MFMA (TY x TX output tiles): w bf16 [Cout][ceil(K*K/4)*16], K = tap*4 + c.
void stem_mfma(const uint8_t* frames, const int32_t* lut_x, const int32_t* lut_y, const bf16* w,
               const float* bias, void* out, int B, int Hc, int Wc, int H, int W, int OH, int OW,
               int Cout, int K, int stride, int act, float out_inv_scale, int TY, int TX,
               hipStream_t s, int mode = 0);
void stem_conv(const uint8_t* frames, const int32_t* lut_x, const int32_t* lut_y, const float* w,
               const float* bias, void* out, int B, int Hc, int Wc, int H, int W, int OH, int OW,
               int Cout, int K, int stride, int act, hipStream_t s, float out_inv_scale = 0.f);

// 3x3 stride-2 pad-1 max pool, NHWC bf16 (ResNet stem).
void maxpool3x3s2(const bf16* in, bf16* out, int B, int IH, int IW, int C, int OH, int OW,
                  hipStream_t s);

// Global average pool NHWC bf16 [B, H, W, C] -> fp32 [B, C]; ws: fp32 workspace of
// gap_workspace_floats(B, C) elements (pixel-slice partial sums).
size_t gap_workspace_floats(int B, int C);
void global_avgpool(const bf16* in, float* out, float* ws, int B, int HW, int C, hipStream_t s);

// out[b, n] = act(sum_k W[n, k] * x[b, k] + bias[n]), fp32 everywhere (tiny).
// out = act(in + bias[n] + img_bias[m / HW][n]) over an [M, N] bf16 matrix (GEMM epilogue)
void bias_act(const bf16* in, const float* bias, const float* img_bias, bf16* out, long long M, int N,
              int HW, int act, hipStream_t s);
void aspp_pool(const bf16* in, float* ws, const float* w1t, const float* b1, const float* w2t,
               float* img_bias, int B, int HW, int C, int N, hipStream_t s, float* dbg = nullptr,
               int mode = 0);
void matvec(const float* x, const float* w, const float* bias, float* out, int B, int N, int K,
            int act, hipStream_t s);

// Bilinear (align_corners=True) upsample of NHWC bf16 logits [B, h, w, ldk]
// (first K channels valid) to H x W, then per-pixel argmax -> uint8 [B, H, W].
// variant: 0 default, 1-4 interval kernels (per-lane / row-block x compare / tagged
// argmax), 5 the direct kernel (see model_ops.hip).
void upsample_argmax(const bf16* logits, uint8_t* labels, int B, int h, int w, int K, int ldk,
                     int H, int W, hipStream_t s, int variant = 0);

// ---- post-processing (postprocess.hip) -------------------------------------
struct PostParams {
  const uint8_t* labels = nullptr;  // [B, H, W] model-resolution label maps
  int B = 0, H = 0, W = 0;          // model resolution (row stride W)
  int crop_h = 0, crop_w = 0;       // letterboxed valid region
  const int32_t* palette = nullptr; // [256, 3] RGB
  int thr = 127;
  double min_area = 0.0;            // pixels^2 (reference: ratio * H * W)
  int num_bins = 32;                // histogram bins (class ids < num_bins)
  int K = 64;                       // record slots per frame
  // workspace (caller-allocated, sizes from post_workspace_bytes)
  void* ws = nullptr;
  float* records = nullptr;         // [B, 1 + 5K] packed output
  int accum = 0;                    // accumulation pass: 0 = pixel strips, 1 / 2 = 32x32 / 64x64 tiles (LDS-staged labels)
};
size_t post_workspace_bytes(int B, int H, int W, int K, int num_bins);

// device buffer -> pinned (hipHostMalloc) host buffer by a kernel on stream s (no host block)
void copy_to_host(const void* src, void* dst, long long nbytes, hipStream_t s);
// dst[r] = [a[r] | b[r]] over `rows` rows of a_words / b_words 4-byte words (a, b: device or
// pinned host memory).
void pack_rows(void* dst, const void* a, int a_words, const void* b, int b_words, int rows,
               hipStream_t s);

void postprocess(const PostParams& p, hipStream_t s);

}  // namespace ssa
