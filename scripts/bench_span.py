"""Microbenchmark + s_memtime phase timeline of the wave-specialised fused IR kernel
(fused_ir_stream) on the 33x33 blocks of DeepLabv3-MobileNetV2 (B = 32, random data and
weights).

  python scripts/bench_span.py [--B 32] [--trace] [--only 16] [--variants 0,1]
"""
import argparse
import sys

import numpy as np
import torch

import os  # noqa: E402
_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
from semantic_segmentation_server_amd.ops import fused_span as FS  # noqa: E402
from test_fused_span_cpu import _block, pack_block  # noqa: E402

BLOCKS = [(7, 64, 64, 1), (10, 64, 96, 1), (11, 96, 96, 1), (13, 96, 160, 1), (14, 160, 160, 2),
          (16, 160, 320, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--H", type=int, default=33)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--only", type=int, default=0, help="run only this block index")
    ap.add_argument("--S", type=int, default=0, help="run only this span count")
    ap.add_argument("--variants", default="", help="comma list of stream variants (default: all)")
    a = ap.parse_args()
    dev = "cuda"
    B, H = a.B, a.H
    for idx, cin, cout, dil in BLOCKS:
        if a.only and idx != a.only:
            continue
        blk, spec = _block(cin, cout, dil, seed=idx)
        packed = pack_block(blk, spec, device=dev)
        x = torch.randn(B, H, H, cin, device=dev).to(torch.bfloat16)
        out = torch.empty(B, H, H, cout, device=dev, dtype=torch.bfloat16)
        flop = 2 * B * H * H * (cin * spec.hidden + spec.hidden * cout + 9 * spec.hidden)
        for S in ((a.S,) if a.S else (8, 16)):
            try:
                tab = FS.span_table(H, H, S, dil, dev)
            except ValueError:
                continue
            opts = ((0, 1, 2) if cout <= 96 and dil == 1 else (0, 1)) + ((4,) if cout <= 160 else ())
            if a.variants:
                opts = tuple(v for v in map(int, a.variants.split(",")) if v in opts)
            if not FS.stream_supported(cin, cout, 1, H, H, S, dil):
                continue
            for npi in opts:
                run = lambda: FS.fused_ir_stream(x, packed, tab, out, B=B, residual=spec.residual, variant=npi)
                for _ in range(3):
                    run()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.reps):
                    run()
                en.record()
                en.synchronize()
                us = st.elapsed_time(en) / a.reps * 1e3
                print(f"block{idx:2d} {cin:3d}->{spec.hidden:3d}->{cout:3d} d{dil} S={S:2d} "
                      f"stream v{npi}: "
                      f"{us:7.1f} us  {flop / us / 1e6:7.1f} TFLOP/s  (xg={tab['xg']}, nh_max={tab['nh_max']})",
                      flush=True)
                if a.trace:
                    tr = torch.zeros(B * S * 2 * 64, dtype=torch.int64, device=dev)
                    FS.fused_ir_stream(x, packed, tab, out, B=B, residual=spec.residual, trace=tr, variant=npi)
                    torch.cuda.synchronize()
                    t = tr.view(B * S, 2, 64).cpu().numpy().astype(np.int64)
                    NC = packed["hidP"] // 32
                    steps = min(NC, 19)
                    for w, role in ((0, "expand"), (1, "dw+proj")):
                        tt = t[:, w]
                        # per step: compute, wait (vmcnt), barrier  (stamps 1 + 3c .. 4 + 3c)
                        ph = np.array([[np.median(tt[:, 2 + 3 * k + i] - tt[:, 1 + 3 * k + i]) for i in range(3)]
                                       for k in range(1, steps - 1)])
                        end = 63 if w == 1 else 1 + 3 * steps
                        print(f"   {role:8s}: prologue {np.median(tt[:, 1] - tt[:, 0]):.0f} cyc; steady step "
                              f"[compute, wait, barrier] = {np.median(ph, axis=0).round(0).tolist()}; "
                              f"step-0 {np.median(tt[:, 4] - tt[:, 1]):.0f}"
                              + (f"; epilogue {np.median(tt[:, 63] - tt[:, 62]):.0f}" if w == 1 else ""),
                              flush=True)


if __name__ == "__main__":
    main()
