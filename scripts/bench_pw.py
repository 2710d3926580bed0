"""Microbenchmark: weight-streamed pw_conv vs the generic conv_gemm on the 1x1 layers
of DeepLabv3-MobileNetV2 (B=32, 513^2, OS16), checked against a torch fp32 reference.

python scripts/bench_pw.py [--reps 20] [--shape NAME]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_server_amd.ops import hip_ops as K  # noqa: E402

# name, M (=B*H*W), Cin, Cout, residual
SHAPES = [
    ("b16_exp", 32 * 33 * 33, 160, 960, False),
    ("b12_exp", 32 * 33 * 33, 96, 576, False),
    ("b8_exp", 32 * 33 * 33, 64, 384, False),
    ("aspp_b0", 32 * 33 * 33, 320, 256, False),
    ("logits", 32 * 33 * 33, 256, 24, False),
    ("b4_exp65", 32 * 65 * 65, 32, 192, False),
    ("b2_exp129", 32 * 129 * 129, 24, 144, False),
    ("b12_proj", 32 * 33 * 33, 576, 96, True),
]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shape", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for name, M, Cin, Cout, resid in SHAPES:
        if a.shape and name != a.shape:
            continue
        if not K.pw_supported(Cin, Cout):
            print(f"{name}: pw unsupported")
            continue
        x = (torch.randn(M, Cin, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(Cout, Cin, device=dev) / Cin ** 0.5).to(torch.bfloat16)
        b = torch.randn(Cout, device=dev)
        res = (torch.randn(M, Cout, device=dev)).to(torch.bfloat16) if resid else None
        act = None if resid else "relu6"
        ref = x.float() @ w.float().t() + b
        if res is not None:
            ref = ref + res.float()
        if act == "relu6":
            ref = ref.clamp(0, 6)
        out = torch.empty(M, Cout, dtype=torch.bfloat16, device=dev)
        us = timeit(lambda: K.conv_gemm(x, w.reshape(Cout, 1, 1, Cin), b, out, B=1, IH=1, IW=M,
                                        Cin=Cin, OH=1, OW=M, Cout=Cout, k=1, act=act, res=res), a.reps)
        err = (out.float() - ref).abs().max().item()
        mb = (M * Cin + M * Cout * (2 if resid else 1)) * 2 / 1e6
        line = [f"{name:10s} M={M:7d} K={Cin:4d} N={Cout:4d} {mb:6.1f}MB  gemm={us:6.1f}us(err {err:.2g})"]
        wpk = K.pack_pw_weights(w, b)
        NC = -(-Cout // 64)
        best = None
        for mt in (2, 4):
            for nch in sorted({1, 2, 3, 5, NC}):
                if nch > NC:
                    continue
                out.zero_()
                us = timeit(lambda: K.pw_conv(x, wpk, out, M=M, K=Cin, N=Cout, act=act, res=res,
                                              mt=mt, nch=nch), a.reps)
                err = (out.float() - ref).abs().max().item()
                line.append(f"pw{mt}/{nch}={us:6.1f}({err:.2g})")
                if best is None or us < best[0]:
                    best = (us, mt, nch)
        line.append(f"best {best[0]:.1f}us {mb / best[0]:.2f}TB/s")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()


def bench_tap(reps=20):
    """ASPP atrous branches: conv_gemm (LDS-DMA, raster / tap-grouped) vs tap_conv."""
    dev = torch.device("cuda")
    B, H, W, Cin, Cout = 32, 33, 33, 320, 256
    x = (torch.randn(B, H, W, Cin, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(Cout, 3, 3, Cin, device=dev) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, device=dev)
    out = torch.empty(B, H, W, 1024, dtype=torch.bfloat16, device=dev)
    wpk, bp = K.pack_tap_weights(w, b)
    for rate in (6, 12, 18):
        ref = out.clone()
        K.conv_gemm(x, w, b, ref, B=B, IH=H, IW=W, Cin=Cin, OH=H, OW=W, Cout=Cout, k=3, dil=rate,
                    ldo=1024, co_off=256, act="relu")
        line = [f"aspp_r{rate}"]
        pg = K.tap_group_perm(B, H, W, 3, rate, 128, dev)
        us = timeit(lambda: K.conv_gemm(x, w, b, out, B=B, IH=H, IW=W, Cin=Cin, OH=H, OW=W, Cout=Cout,
                                        k=3, dil=rate, ldo=1024, co_off=256, act="relu", variant=4,
                                        perm=pg), reps)
        line.append(f"gemm_v4g={us:6.1f}")
        for grouped in (False, True):
            perm = K.tap_group_perm(B, H, W, 3, rate, 256, dev) if grouped else None
            out.zero_()
            us = timeit(lambda: K.tap_conv(x, wpk, bp, out, B=B, H=H, W=W, Cin=Cin, Cout=Cout, k=3,
                                           dil=rate, ldo=1024, co_off=256, act="relu", perm=perm), reps)
            err = (out[..., 256:512].float() - ref[..., 256:512].float()).abs().max().item()
            line.append(f"tap{'g' if grouped else ''}={us:6.1f}({err:.2g})")
        print("  ".join(line), flush=True)


if __name__ == "__main__" and os.environ.get("SSA_BENCH_TAP", "1") == "1":
    bench_tap()
