"""Microbenchmark of the conv_gemm variants on the models' real layer shapes.

python scripts/bench_conv.py [--reps 20] [--only mnv2|r50]  -> one line per (shape, variant):
time (us), effective TFLOP/s (nominal MACs incl. padding taps), max |diff| vs variant 2.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_server_amd.ops import hip_ops as K  # noqa: E402

SHAPES = {
    "mnv2": [  # B=32, 513^2 input, OS16 -> 33x33 maps
        ("aspp_r6", 32, 33, 33, 320, 256, 3, 1, 6),
        ("aspp_r12", 32, 33, 33, 320, 256, 3, 1, 12),
        ("aspp_r18", 32, 33, 33, 320, 256, 3, 1, 18),
        ("aspp_proj", 32, 33, 33, 768, 256, 1, 1, 1),
        ("aspp_b0", 32, 33, 33, 320, 256, 1, 1, 1),
        ("b17_proj", 32, 33, 33, 960, 320, 1, 1, 1),
        ("b15_proj", 32, 33, 33, 960, 160, 1, 1, 1),
        ("b15_exp", 32, 33, 33, 160, 960, 1, 1, 1),
        ("b12_proj", 32, 33, 33, 576, 96, 1, 1, 1),
    ],
    "r50": [  # B=8, 1025^2 input, OS16
        ("l1_c1", 8, 257, 257, 256, 64, 1, 1, 1),
        ("l1_c2", 8, 257, 257, 64, 64, 3, 1, 1),
        ("l1_c3", 8, 257, 257, 64, 256, 1, 1, 1),
        ("l2_c2", 8, 129, 129, 128, 128, 3, 1, 1),
        ("l2_c3", 8, 129, 129, 128, 512, 1, 1, 1),
        ("l3_c1", 8, 65, 65, 1024, 256, 1, 1, 1),
        ("l3_c2", 8, 65, 65, 256, 256, 3, 1, 1),
        ("l3_c3", 8, 65, 65, 256, 1024, 1, 1, 1),
        ("l4_c1", 8, 65, 65, 2048, 512, 1, 1, 1),
        ("l4_c2", 8, 65, 65, 512, 512, 3, 1, 2),
        ("l4_c3", 8, 65, 65, 512, 2048, 1, 1, 1),
        ("aspp_r12", 8, 65, 65, 2048, 256, 3, 1, 12),
        ("aspp_proj", 8, 65, 65, 1024, 256, 1, 1, 1),
    ],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--variants", default="1,4,5,6")
    ap.add_argument("--shape", default=None, help="only this shape name (e.g. b15_exp)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    variants = [int(v) for v in a.variants.split(",")]
    for fam, shapes in SHAPES.items():
        if a.only and fam != a.only:
            continue
        for name, B, H, W, Cin, Cout, k, stride, dil in shapes:
            if a.shape and name != a.shape:
                continue
            OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
            x = (torch.randn(B, H, W, Cin, device=dev) * 0.5).to(torch.bfloat16)
            w = (torch.randn(Cout, k, k, Cin, device=dev) / (Cin * k * k) ** 0.5).to(torch.bfloat16)
            b = torch.randn(Cout, device=dev)
            macs = B * OH * OW * Cout * Cin * k * k
            ref = None
            line = [f"{fam}/{name:10s} M={B*OH*OW:7d} N={Cout:5d} K={Cin*k*k:6d}"]
            for v in variants:
                out = torch.empty(B, OH, OW, Cout, dtype=torch.bfloat16, device=dev)
                run = lambda: K.conv_gemm(x, w, b, out, B=B, IH=H, IW=W, Cin=Cin, OH=OH, OW=OW,
                                          Cout=Cout, k=k, stride=stride, dil=dil, act="relu",
                                          variant=v)
                for _ in range(3):
                    run()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.reps):
                    run()
                en.record()
                torch.cuda.synchronize()
                us = st.elapsed_time(en) * 1e3 / a.reps
                if ref is None:
                    ref = out.float()
                    err = 0.0
                else:
                    err = (out.float() - ref).abs().max().item()
                line.append(f"v{v}={us:7.1f}us/{2 * macs / us / 1e6:6.0f}TF(err {err:.2g})")
            print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
