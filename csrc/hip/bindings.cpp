// pybind11 bindings of the gfx950 kernels (module: _hip). Arguments are raw
// device pointers (Python ints from tensor.data_ptr()) and a HIP stream handle
// (torch.cuda.current_stream().cuda_stream), so every launch lands on the
// caller's stream and is captured by an enclosing hipGraph capture. Shape checks
// live in the Python wrappers (semantic_segmentation_server_amd/ops/hip_ops.py).
#include <pybind11/pybind11.h>

#include <vector>

#include "kernels.h"

namespace py = pybind11;
using namespace ssa;

namespace {
template <class T>
T* P(uintptr_t v) { return reinterpret_cast<T*>(v); }
hipStream_t S(uintptr_t v) { return reinterpret_cast<hipStream_t>(v); }
}  // namespace

PYBIND11_MODULE(_hip, m) {
  m.doc() = "gfx950 HIP kernels for DeepLabv3 inference and contour statistics";

  m.def("conv_gemm",
        [](uintptr_t in, uintptr_t w, uintptr_t bias, uintptr_t img_bias, uintptr_t res,
           uintptr_t out, int B, int IH, int IW, int Cin, int OH, int OW, int Cout, int KH, int KW,
           int stride, int dil, int ldo, int co_off, int ldr, int act, uintptr_t stream, int variant,
           uintptr_t perm, int Mp) {
          ConvParams p;
          p.perm = P<const int>(perm); p.Mp = Mp;
          p.in = P<const bf16>(in); p.w = P<const bf16>(w); p.bias = P<const float>(bias);
          p.img_bias = P<const float>(img_bias); p.res = P<const bf16>(res); p.out = P<bf16>(out);
          p.B = B; p.IH = IH; p.IW = IW; p.Cin = Cin; p.OH = OH; p.OW = OW; p.Cout = Cout;
          p.KH = KH; p.KW = KW; p.stride = stride; p.dil = dil; p.ldo = ldo; p.co_off = co_off;
          p.ldr = ldr; p.act = act; p.variant = variant;
          conv_gemm(p, S(stream));
        },
        py::arg("in"), py::arg("w"), py::arg("bias"), py::arg("img_bias"), py::arg("res"),
        py::arg("out"), py::arg("B"), py::arg("IH"), py::arg("IW"), py::arg("Cin"), py::arg("OH"),
        py::arg("OW"), py::arg("Cout"), py::arg("KH"), py::arg("KW"), py::arg("stride"),
        py::arg("dil"), py::arg("ldo"), py::arg("co_off"), py::arg("ldr"), py::arg("act"),
        py::arg("stream"), py::arg("variant") = 0, py::arg("perm") = 0, py::arg("Mp") = 0);

  m.def("conv_gemm_grouped",
        [](py::list groups, uintptr_t order, int nblocks, int variant, uintptr_t stream, int ks, uintptr_t part,
           uintptr_t cnt, int cnt_stride) {
          // groups: tuples (in, w, bias, img_bias, res, out, B, IH, IW, Cin, OH, OW, Cout,
          //                 KH, KW, stride, dil, ldo, co_off, ldr, act, perm, Mp)
          std::vector<ConvParams> ps;
          for (auto item : groups) {
            auto t = item.cast<py::tuple>();
            if (t.size() != 23) throw std::invalid_argument("conv_gemm_grouped: 23-tuple per conv");
            auto I = [&](int i) { return t[i].cast<int>(); };
            auto U = [&](int i) { return t[i].cast<uintptr_t>(); };
            ConvParams p;
            p.in = P<const bf16>(U(0)); p.w = P<const bf16>(U(1)); p.bias = P<const float>(U(2));
            p.img_bias = P<const float>(U(3)); p.res = P<const bf16>(U(4)); p.out = P<bf16>(U(5));
            p.B = I(6); p.IH = I(7); p.IW = I(8); p.Cin = I(9); p.OH = I(10); p.OW = I(11);
            p.Cout = I(12); p.KH = I(13); p.KW = I(14); p.stride = I(15); p.dil = I(16);
            p.ldo = I(17); p.co_off = I(18); p.ldr = I(19); p.act = I(20);
            p.perm = P<const int>(U(21)); p.Mp = I(22);
            ps.push_back(p);
          }
          conv_gemm_grouped(ps.data(), (int)ps.size(), P<const int>(order), nblocks, variant,
                            S(stream), ks, P<float>(part), P<int>(cnt), cnt_stride);
        },
        py::arg("groups"), py::arg("order"), py::arg("nblocks"), py::arg("variant"),
        py::arg("stream"), py::arg("ks") = 1, py::arg("part") = 0, py::arg("cnt") = 0,
        py::arg("cnt_stride") = 0);

  m.def("bias_act", [](uintptr_t in, uintptr_t bias, uintptr_t img_bias, uintptr_t out, long long M,
                       int N, int HW, int act, uintptr_t stream) {
    bias_act(P<const bf16>(in), P<const float>(bias), P<const float>(img_bias), P<bf16>(out), M, N, HW,
             act, S(stream));
  });

  m.def("fused_ir",
        [](uintptr_t in, uintptr_t we, uintptr_t be, uintptr_t wd, uintptr_t bd, uintptr_t wp,
           uintptr_t bp, uintptr_t out, int B, int IH, int IW, int Cin, int CinP, int hidP,
           int Cout, int OH, int OW, int stride, int residual, uintptr_t stream, int dil, int TY,
           int TX, uintptr_t wd_h, uintptr_t bd_h, uintptr_t wp_h, uintptr_t trace) {
          FusedIRParams p;
          p.in = P<const bf16>(in); p.we = P<const bf16>(we); p.be = P<const float>(be);
          p.wd = P<const float>(wd); p.bd = P<const float>(bd); p.wp = P<const bf16>(wp);
          p.bp = P<const float>(bp); p.out = P<bf16>(out);
          p.B = B; p.IH = IH; p.IW = IW; p.Cin = Cin; p.CinP = CinP; p.hidP = hidP; p.Cout = Cout;
          p.OH = OH; p.OW = OW; p.stride = stride; p.residual = residual;
          p.dil = dil; p.TY = TY; p.TX = TX;
          p.wd_h = P<const void>(wd_h); p.bd_h = P<const void>(bd_h); p.wp_h = P<const void>(wp_h);
          p.trace = P<long long>(trace);
          fused_inverted_residual(p, S(stream));
        },
        py::arg("in"), py::arg("we"), py::arg("be"), py::arg("wd"), py::arg("bd"), py::arg("wp"),
        py::arg("bp"), py::arg("out"), py::arg("B"), py::arg("IH"), py::arg("IW"), py::arg("Cin"),
        py::arg("CinP"), py::arg("hidP"), py::arg("Cout"), py::arg("OH"), py::arg("OW"),
        py::arg("stride"), py::arg("residual"), py::arg("stream"), py::arg("dil") = 1,
        py::arg("TY") = 0, py::arg("TX") = 0, py::arg("wd_h") = 0, py::arg("bd_h") = 0,
        py::arg("wp_h") = 0, py::arg("trace") = 0);
  m.def("fused_ir_stream",
        [](uintptr_t in, uintptr_t w, uintptr_t bp, uintptr_t table, uintptr_t out, int B, int H,
           int W, int Cin, int hidP, int Cout, int dil, int residual, int nspan, int WR, int WCP,
           int hstride, int nh_max, uintptr_t stream, uintptr_t trace, int variant, int hsplit,
           uintptr_t part, uintptr_t cnt) {
          FusedSpanParams p;
          p.trace = P<long long>(trace);
          p.hsplit = hsplit;
          p.part = P<float>(part);
          p.cnt = P<int>(cnt);
          p.npi = variant;  // 0: 8 waves; 1: group 8 on the expansion waves (G8A); 2: 12 waves
          p.in = P<const bf16>(in); p.w = P<const void>(w); p.bp = P<const float>(bp);
          p.table = P<const int>(table); p.out = P<bf16>(out);
          p.B = B; p.H = H; p.W = W; p.Cin = Cin; p.hidP = hidP; p.Cout = Cout; p.dil = dil;
          p.residual = residual; p.S = nspan; p.WR = WR; p.WCP = WCP; p.hstride = hstride;
          p.nh_max = nh_max;
          fused_ir_stream(p, S(stream));
        },
        py::arg("in"), py::arg("w"), py::arg("bp"), py::arg("table"), py::arg("out"), py::arg("B"),
        py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("hidP"), py::arg("Cout"), py::arg("dil"),
        py::arg("residual"), py::arg("nspan"), py::arg("WR"), py::arg("WCP"), py::arg("hstride"),
        py::arg("nh_max"), py::arg("stream"), py::arg("trace") = 0, py::arg("variant") = 0,
        py::arg("hsplit") = 1, py::arg("part") = 0, py::arg("cnt") = 0);
  m.def("fused_ir_stream_lds", &fused_ir_stream_lds, py::arg("Cin"), py::arg("Cout"), py::arg("WR"),
        py::arg("WCP"), py::arg("nsl") = 0);
  m.def("stream_combine",
        [](uintptr_t part, uintptr_t bp, uintptr_t res, uintptr_t out, int HS, long long M, int Cout,
           uintptr_t stream, int act) {
          stream_combine(P<const float>(part), P<const float>(bp), P<const bf16>(res), P<bf16>(out), HS, M, Cout,
                         S(stream), act);
        },
        py::arg("part"), py::arg("bp"), py::arg("res"), py::arg("out"), py::arg("HS"), py::arg("M"),
        py::arg("Cout"), py::arg("stream"), py::arg("act") = 0);
  m.def("fused_ir_band",
        [](uintptr_t in, uintptr_t blob, uintptr_t out, int B, int IH, int IW, int Cin, int OH, int OW,
           int Cout, int hidP, int stride, int residual, int R, int nslot, int blob_bytes, int o_be,
           int o_wd, int o_bd, int o_wp, int o_bp, uintptr_t stream, int hs, int split) {
          FusedBandParams p;
          p.hs = hs;
          p.split = split;
          p.in = P<const bf16>(in); p.blob = P<const void>(blob); p.out = P<bf16>(out);
          p.B = B; p.IH = IH; p.IW = IW; p.Cin = Cin; p.OH = OH; p.OW = OW; p.Cout = Cout;
          p.hidP = hidP; p.stride = stride; p.residual = residual; p.R = R; p.nslot = nslot;
          p.blob_bytes = blob_bytes; p.o_be = o_be; p.o_wd = o_wd; p.o_bd = o_bd; p.o_wp = o_wp;
          p.o_bp = o_bp;
          fused_ir_band(p, S(stream));
        },
        py::arg("in"), py::arg("blob"), py::arg("out"), py::arg("B"), py::arg("IH"), py::arg("IW"),
        py::arg("Cin"), py::arg("OH"), py::arg("OW"), py::arg("Cout"), py::arg("hidP"), py::arg("stride"),
        py::arg("residual"), py::arg("R"), py::arg("nslot"), py::arg("blob_bytes"), py::arg("o_be"),
        py::arg("o_wd"), py::arg("o_bd"), py::arg("o_wp"), py::arg("o_bp"), py::arg("stream"),
        py::arg("hs") = 1, py::arg("split") = 1);
  m.def("fused_ir_slice",
        [](uintptr_t in, uintptr_t blob, uintptr_t out, int B, int IH, int IW, int Cin, int OH, int OW,
           int Cout, int hidP, int stride, int residual, int R, int o_be, int o_wd, int o_bd, int o_wp,
           int o_bp, int nw, uintptr_t stream, int one_barrier) {
          FusedBandParams p;
          p.in = P<const bf16>(in); p.blob = P<const void>(blob); p.out = P<bf16>(out);
          p.B = B; p.IH = IH; p.IW = IW; p.Cin = Cin; p.OH = OH; p.OW = OW; p.Cout = Cout;
          p.hidP = hidP; p.stride = stride; p.residual = residual; p.R = R;
          p.o_be = o_be; p.o_wd = o_wd; p.o_bd = o_bd; p.o_wp = o_wp; p.o_bp = o_bp;
          fused_ir_slice(p, nw, S(stream), one_barrier != 0);
        },
        py::arg("in"), py::arg("blob"), py::arg("out"), py::arg("B"), py::arg("IH"), py::arg("IW"),
        py::arg("Cin"), py::arg("OH"), py::arg("OW"), py::arg("Cout"), py::arg("hidP"), py::arg("stride"),
        py::arg("residual"), py::arg("R"), py::arg("o_be"), py::arg("o_wd"), py::arg("o_bd"),
        py::arg("o_wp"), py::arg("o_bp"), py::arg("nw"), py::arg("stream"), py::arg("one_barrier") = 0);
  m.def("fused_ir_slice_lds", &fused_ir_slice_lds, py::arg("stride"), py::arg("hidP"), py::arg("OW"),
        py::arg("Cout"), py::arg("nw"), py::arg("one_barrier") = false);
  m.def("fused_ir_band_lds", &fused_ir_band_lds, py::arg("stride"), py::arg("hidP"), py::arg("OW"),
        py::arg("blob_bytes"), py::arg("nslot"), py::arg("hs") = 1, py::arg("Cout") = 0,
        py::arg("split") = 1);
  m.def("fused_ir_tile_lds", &fused_ir_tile_lds);
  m.def("stem_block0",
        [](uintptr_t frames, uintptr_t lx, uintptr_t ly, uintptr_t ws, uintptr_t bs, uintptr_t wd,
           uintptr_t bd, uintptr_t wp, uintptr_t bp, uintptr_t out, int B, int Hc, int Wc, int H,
           int W, int SH, int SW, int Cout, int TY, int TX, uintptr_t stream) {
          StemBlock0Params p;
          p.frames = P<const uint8_t>(frames); p.lut_x = P<const int32_t>(lx); p.lut_y = P<const int32_t>(ly);
          p.ws = P<const bf16>(ws); p.bs = P<const float>(bs); p.wd = P<const void>(wd);
          p.bd = P<const void>(bd); p.wp = P<const void>(wp); p.bp = P<const float>(bp); p.out = P<bf16>(out);
          p.B = B; p.Hc = Hc; p.Wc = Wc; p.H = H; p.W = W; p.SH = SH; p.SW = SW; p.Cout = Cout;
          p.TY = TY; p.TX = TX;
          stem_block0(p, S(stream));
        });
  m.def("stem_band",
        [](uintptr_t frames, uintptr_t lx, uintptr_t ly, uintptr_t ws, uintptr_t bs, uintptr_t wd,
           uintptr_t bd, uintptr_t wp, uintptr_t bp, uintptr_t out, int B, int Hc, int Wc, int H,
           int W, int SH, int SW, int R, int nbx, uintptr_t stream, int one_barrier) {
          StemBlock0Params p;
          p.frames = P<const uint8_t>(frames); p.lut_x = P<const int32_t>(lx); p.lut_y = P<const int32_t>(ly);
          p.ws = P<const bf16>(ws); p.bs = P<const float>(bs); p.wd = P<const void>(wd);
          p.bd = P<const void>(bd); p.wp = P<const void>(wp); p.bp = P<const float>(bp); p.out = P<bf16>(out);
          p.B = B; p.Hc = Hc; p.Wc = Wc; p.H = H; p.W = W; p.SH = SH; p.SW = SW; p.Cout = 16;
          p.TY = R;
          stem_band(p, nbx, S(stream), one_barrier != 0);
        },
        py::arg("frames"), py::arg("lx"), py::arg("ly"), py::arg("ws"), py::arg("bs"), py::arg("wd"),
        py::arg("bd"), py::arg("wp"), py::arg("bp"), py::arg("out"), py::arg("B"), py::arg("Hc"),
        py::arg("Wc"), py::arg("H"), py::arg("W"), py::arg("SH"), py::arg("SW"), py::arg("R"),
        py::arg("nbx"), py::arg("stream"), py::arg("one_barrier") = 1);
  m.def("stem_band_lds", &stem_band_lds, py::arg("SW"), py::arg("nbx"), py::arg("R"));

  m.def("aspp_head",
        [](uintptr_t cat, uintptr_t wp, uintptr_t bp, uintptr_t img_bias, uintptr_t wl, uintptr_t bl,
           uintptr_t out, int M, int K, int HW, int ncls, int ldo, int G, uintptr_t stream, int waves) {
          AsppHeadParams p;
          p.waves = waves;
          p.cat = P<const bf16>(cat); p.wp = P<const bf16>(wp); p.bp = P<const float>(bp);
          p.img_bias = P<const float>(img_bias); p.wl = P<const bf16>(wl); p.bl = P<const float>(bl);
          p.out = P<bf16>(out);
          p.M = M; p.K = K; p.HW = HW; p.ncls = ncls; p.ldo = ldo; p.G = G;
          aspp_head(p, S(stream));
        },
        py::arg("cat"), py::arg("wp"), py::arg("bp"), py::arg("img_bias"), py::arg("wl"), py::arg("bl"),
        py::arg("out"), py::arg("M"), py::arg("K"), py::arg("HW"), py::arg("ncls"), py::arg("ldo"),
        py::arg("G"), py::arg("stream"), py::arg("waves") = 8);

  m.def("dw_project",
        [](uintptr_t hid_in, uintptr_t wd, uintptr_t bd, uintptr_t wp, uintptr_t bp, uintptr_t res,
           uintptr_t out, int B, int IH, int IW, int hid, int Cout, int OH, int OW, int stride,
           int dil, uintptr_t stream) {
          DwProjectParams p;
          p.hid_in = P<const bf16>(hid_in); p.wd = P<const float>(wd); p.bd = P<const float>(bd);
          p.wp = P<const bf16>(wp); p.bp = P<const float>(bp); p.res = P<const bf16>(res);
          p.out = P<bf16>(out);
          p.B = B; p.IH = IH; p.IW = IW; p.hid = hid; p.Cout = Cout; p.OH = OH; p.OW = OW;
          p.stride = stride; p.dil = dil;
          dw_project(p, S(stream));
        });

  m.def("dw_proj_fused",
        [](uintptr_t h, uintptr_t w, uintptr_t bp, uintptr_t res, uintptr_t out, int B, int IH,
           int IW, int hid, int Cout, int OH, int OW, int stride, int dil, int waves,
           uintptr_t stream, int rows) {
          DwProjFusedParams p;
          p.rows = rows;
          p.h = P<const void>(h); p.w = P<const void>(w); p.bp = P<const float>(bp);
          p.res = P<const bf16>(res); p.out = P<bf16>(out);
          p.B = B; p.IH = IH; p.IW = IW; p.hid = hid; p.Cout = Cout; p.OH = OH; p.OW = OW;
          p.stride = stride; p.dil = dil; p.waves = waves;
          dw_proj_fused(p, S(stream));
        },
        py::arg("h"), py::arg("w"), py::arg("bp"), py::arg("res"), py::arg("out"), py::arg("B"),
        py::arg("IH"), py::arg("IW"), py::arg("hid"), py::arg("Cout"), py::arg("OH"), py::arg("OW"),
        py::arg("stride"), py::arg("dil"), py::arg("waves"), py::arg("stream"), py::arg("rows") = 0);

  m.def("depthwise3x3",
        [](uintptr_t in, uintptr_t w, uintptr_t bias, uintptr_t out, int B, int IH, int IW, int C,
           int OH, int OW, int stride, int dil, int act, uintptr_t stream) {
          depthwise3x3(P<const bf16>(in), P<const float>(w), P<const float>(bias), P<bf16>(out), B,
                       IH, IW, C, OH, OW, stride, dil, act, S(stream));
        });

  m.def("stem_mfma",
        [](uintptr_t frames, uintptr_t lut_x, uintptr_t lut_y, uintptr_t w, uintptr_t bias,
           uintptr_t out, int B, int Hc, int Wc, int H, int W, int OH, int OW, int Cout, int K,
           int stride, int act, float out_inv_scale, int TY, int TX, uintptr_t stream, int mode) {
          stem_mfma(P<const uint8_t>(frames), P<const int32_t>(lut_x), P<const int32_t>(lut_y),
                    P<const bf16>(w), P<const float>(bias), P<void>(out), B, Hc, Wc, H, W, OH, OW,
                    Cout, K, stride, act, out_inv_scale, TY, TX, S(stream), mode);
        }, py::arg("frames"), py::arg("lut_x"), py::arg("lut_y"), py::arg("w"), py::arg("bias"),
        py::arg("out"), py::arg("B"), py::arg("Hc"), py::arg("Wc"), py::arg("H"), py::arg("W"),
        py::arg("OH"), py::arg("OW"), py::arg("Cout"), py::arg("K"), py::arg("stride"), py::arg("act"),
        py::arg("out_inv_scale"), py::arg("TY"), py::arg("TX"), py::arg("stream"), py::arg("mode") = 0);
  m.def("stem_conv",
        [](uintptr_t frames, uintptr_t lut_x, uintptr_t lut_y, uintptr_t w, uintptr_t bias,
           uintptr_t out, int B, int Hc, int Wc, int H, int W, int OH, int OW, int Cout, int K,
           int stride, int act, uintptr_t stream, float out_inv_scale) {
          stem_conv(P<const uint8_t>(frames), P<const int32_t>(lut_x), P<const int32_t>(lut_y),
                    P<const float>(w), P<const float>(bias), P<void>(out), B, Hc, Wc, H, W, OH, OW,
                    Cout, K, stride, act, S(stream), out_inv_scale);
        },
        py::arg("frames"), py::arg("lut_x"), py::arg("lut_y"), py::arg("w"), py::arg("bias"),
        py::arg("out"), py::arg("B"), py::arg("Hc"), py::arg("Wc"), py::arg("H"), py::arg("W"),
        py::arg("OH"), py::arg("OW"), py::arg("Cout"), py::arg("K"), py::arg("stride"),
        py::arg("act"), py::arg("stream"), py::arg("out_inv_scale") = 0.f);

  m.def("pw_conv",
        [](uintptr_t in, uintptr_t w, uintptr_t img_bias, uintptr_t res,
           uintptr_t out, int M, int K, int N, int HW, int ldo, int co_off, int ldr, int act,
           int mt, int nch, uintptr_t stream, int out_f16) {
          PwConvParams p;
          p.out_f16 = out_f16;
          p.in = P<const bf16>(in); p.w = P<const bf16>(w);
          p.img_bias = P<const float>(img_bias); p.res = P<const bf16>(res); p.out = P<bf16>(out);
          p.M = M; p.K = K; p.N = N; p.HW = HW; p.ldo = ldo; p.co_off = co_off; p.ldr = ldr;
          p.act = act; p.mt = mt; p.nch = nch;
          pw_conv(p, S(stream));
        },
        py::arg("in"), py::arg("w"), py::arg("img_bias"), py::arg("res"), py::arg("out"),
        py::arg("M"), py::arg("K"), py::arg("N"), py::arg("HW"), py::arg("ldo"), py::arg("co_off"),
        py::arg("ldr"), py::arg("act"), py::arg("mt"), py::arg("nch"), py::arg("stream"),
        py::arg("out_f16") = 0);
  m.def("pw_conv_supported_ks", &pw_conv_supported_ks);
  m.def("tap_conv",
        [](uintptr_t in, uintptr_t w, uintptr_t bias, uintptr_t out, uintptr_t perm, int Mp, int B,
           int H, int W, int Cin, int Cout, int KH, int KW, int dil, int ldo, int co_off, int act,
           uintptr_t stream) {
          TapConvParams p;
          p.in = P<const bf16>(in); p.w = P<const bf16>(w); p.bias = P<const float>(bias);
          p.out = P<bf16>(out); p.perm = P<const int>(perm); p.Mp = Mp;
          p.B = B; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout; p.KH = KH; p.KW = KW;
          p.dil = dil; p.ldo = ldo; p.co_off = co_off; p.act = act;
          tap_conv(p, S(stream));
        });
  m.def("tap_conv_group_channels", &tap_conv_group_channels);

  m.def("conv_i8",
        [](uintptr_t in, uintptr_t w, uintptr_t scale, uintptr_t bias, uintptr_t img_bias,
           uintptr_t res, float res_scale, uintptr_t out, float inv_out_scale, int out_mode, int B,
           int IH, int IW, int Cin, int OH, int OW, int Cout, int KH, int KW, int stride, int dil,
           int ldo, int co_off, int act, uintptr_t stream, int variant, uintptr_t perm, int Mp) {
          ConvI8Params p;
          p.variant = variant;
          p.perm = P<const int>(perm); p.Mp = Mp;
          p.in = P<const int8_t>(in); p.w = P<const int8_t>(w); p.scale = P<const float>(scale);
          p.bias = P<const float>(bias); p.img_bias = P<const float>(img_bias);
          p.res = P<const int8_t>(res); p.res_scale = res_scale; p.out = P<void>(out);
          p.inv_out_scale = inv_out_scale; p.out_mode = out_mode;
          p.B = B; p.IH = IH; p.IW = IW; p.Cin = Cin; p.OH = OH; p.OW = OW; p.Cout = Cout;
          p.KH = KH; p.KW = KW; p.stride = stride; p.dil = dil; p.ldo = ldo; p.co_off = co_off;
          p.act = act;
          conv_i8(p, S(stream));
        },
        py::arg("in"), py::arg("w"), py::arg("scale"), py::arg("bias"), py::arg("img_bias"),
        py::arg("res"), py::arg("res_scale"), py::arg("out"), py::arg("inv_out_scale"),
        py::arg("out_mode"), py::arg("B"), py::arg("IH"), py::arg("IW"), py::arg("Cin"),
        py::arg("OH"), py::arg("OW"), py::arg("Cout"), py::arg("KH"), py::arg("KW"),
        py::arg("stride"), py::arg("dil"), py::arg("ldo"), py::arg("co_off"), py::arg("act"),
        py::arg("stream"), py::arg("variant") = 0, py::arg("perm") = 0, py::arg("Mp") = 0);
  m.def("conv_i8_grouped",
        [](py::list groups, uintptr_t order, int nblocks, int variant, uintptr_t stream) {
          // groups: tuples (in, w, scale, bias, img_bias, res, res_scale, out, inv_out_scale,
          //                 out_mode, B, IH, IW, Cin, OH, OW, Cout, KH, KW, stride, dil, ldo,
          //                 co_off, act, perm, Mp)
          std::vector<ConvI8Params> ps;
          for (auto item : groups) {
            auto t = item.cast<py::tuple>();
            if (t.size() != 26) throw std::invalid_argument("conv_i8_grouped: 26-tuple per conv");
            auto I = [&](int i) { return t[i].cast<int>(); };
            auto U = [&](int i) { return t[i].cast<uintptr_t>(); };
            ConvI8Params p;
            p.in = P<const int8_t>(U(0)); p.w = P<const int8_t>(U(1)); p.scale = P<const float>(U(2));
            p.bias = P<const float>(U(3)); p.img_bias = P<const float>(U(4)); p.res = P<const int8_t>(U(5));
            p.res_scale = t[6].cast<float>(); p.out = P<void>(U(7)); p.inv_out_scale = t[8].cast<float>();
            p.out_mode = I(9); p.B = I(10); p.IH = I(11); p.IW = I(12); p.Cin = I(13); p.OH = I(14);
            p.OW = I(15); p.Cout = I(16); p.KH = I(17); p.KW = I(18); p.stride = I(19); p.dil = I(20);
            p.ldo = I(21); p.co_off = I(22); p.act = I(23); p.perm = P<const int>(U(24)); p.Mp = I(25);
            ps.push_back(p);
          }
          conv_i8_grouped(ps.data(), (int)ps.size(), P<const int>(order), nblocks, variant, S(stream));
        },
        py::arg("groups"), py::arg("order"), py::arg("nblocks"), py::arg("variant"), py::arg("stream"));
  m.def("maxpool3x3s2_i8", [](uintptr_t in, uintptr_t out, int B, int IH, int IW, int C, int OH,
                              int OW, uintptr_t stream) {
    maxpool3x3s2_i8(P<const int8_t>(in), P<int8_t>(out), B, IH, IW, C, OH, OW, S(stream));
  });
  m.def("global_avgpool_i8", [](uintptr_t in, uintptr_t out, uintptr_t ws, int B, int HW, int C,
                                float scale, uintptr_t stream) {
    global_avgpool_i8(P<const int8_t>(in), P<float>(out), P<float>(ws), B, HW, C, scale, S(stream));
  });

  m.def("maxpool3x3s2", [](uintptr_t in, uintptr_t out, int B, int IH, int IW, int C, int OH,
                           int OW, uintptr_t stream) {
    maxpool3x3s2(P<const bf16>(in), P<bf16>(out), B, IH, IW, C, OH, OW, S(stream));
  });

  m.def("gap_workspace_floats", &gap_workspace_floats);
  m.def("global_avgpool", [](uintptr_t in, uintptr_t out, uintptr_t ws, int B, int HW, int C,
                             uintptr_t stream) {
    global_avgpool(P<const bf16>(in), P<float>(out), P<float>(ws), B, HW, C, S(stream));
  });

  m.def("matvec", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t out, int B, int N, int K,
                     int act, uintptr_t stream) {
    matvec(P<const float>(x), P<const float>(w), P<const float>(bias), P<float>(out), B, N, K, act,
           S(stream));
  });

  m.def("aspp_pool", [](uintptr_t in, uintptr_t ws, uintptr_t w1t, uintptr_t b1, uintptr_t w2t,
                        uintptr_t img_bias, int B, int HW, int C, int N, uintptr_t stream,
                        uintptr_t dbg, int mode) {
    aspp_pool(P<const bf16>(in), P<float>(ws), P<const float>(w1t), P<const float>(b1), P<const float>(w2t),
              P<float>(img_bias), B, HW, C, N, S(stream), P<float>(dbg), mode);
  }, py::arg("in"), py::arg("ws"), py::arg("w1t"), py::arg("b1"), py::arg("w2t"), py::arg("img_bias"),
     py::arg("B"), py::arg("HW"), py::arg("C"), py::arg("N"), py::arg("stream"), py::arg("dbg") = 0,
     py::arg("mode") = 0);

  m.def("upsample_argmax", [](uintptr_t logits, uintptr_t labels, int B, int h, int w, int K,
                              int ldk, int H, int W, uintptr_t stream, int variant) {
    upsample_argmax(P<const bf16>(logits), P<uint8_t>(labels), B, h, w, K, ldk, H, W, S(stream),
                    variant);
  });

  m.def("post_workspace_bytes", &post_workspace_bytes);
  m.def("copy_to_host", [](uintptr_t src, uintptr_t dst, long long nbytes, uintptr_t stream) {
    copy_to_host(P<const void>(src), P<void>(dst), nbytes, S(stream));
  });
  m.def("pack_rows", [](uintptr_t dst, uintptr_t a, int aw, uintptr_t b, int bw, int rows,
                        uintptr_t stream) {
    pack_rows(P<void>(dst), P<const void>(a), aw, P<const void>(b), bw, rows, S(stream));
  });
  m.def("postprocess",
        [](uintptr_t labels, int B, int H, int W, int crop_h, int crop_w, uintptr_t palette,
           int thr, double min_area, int num_bins, int K, uintptr_t ws, uintptr_t records,
           uintptr_t stream, int accum) {
          PostParams p;
          p.accum = accum;
          p.labels = P<const uint8_t>(labels); p.B = B; p.H = H; p.W = W;
          p.crop_h = crop_h; p.crop_w = crop_w; p.palette = P<const int32_t>(palette);
          p.thr = thr; p.min_area = min_area; p.num_bins = num_bins; p.K = K;
          p.ws = P<void>(ws); p.records = P<float>(records);
          postprocess(p, S(stream));
        },
        py::arg("labels"), py::arg("B"), py::arg("H"), py::arg("W"), py::arg("crop_h"), py::arg("crop_w"),
        py::arg("palette"), py::arg("thr"), py::arg("min_area"), py::arg("num_bins"), py::arg("K"),
        py::arg("ws"), py::arg("records"), py::arg("stream"), py::arg("accum") = 0);

  m.attr("ACT_NONE") = (int)ACT_NONE;
  m.attr("ACT_RELU") = (int)ACT_RELU;
  m.attr("ACT_RELU6") = (int)ACT_RELU6;
}
