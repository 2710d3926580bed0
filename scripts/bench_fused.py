"""Time the fused inverted-residual variants on one MobileNetV2 block shape (B=32, 513 input).

python scripts/bench_fused.py --block 14 [--reps 20] [--tiles 5x11,11x11]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_server_amd.models.layers import init_random  # noqa: E402
from semantic_segmentation_server_amd.models.mobilenetv2 import (InvertedResidual,  # noqa: E402
                                                                  mnv2_block_specs)
from semantic_segmentation_server_amd.ops import hip_ops as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--block", type=int, default=14)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--tiles", default="5x11,11x11,8x16")
    ap.add_argument("--trace", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    _, specs = mnv2_block_specs(1.0, 16)
    sp = specs[a.block]
    H = {0: 257, 1: 257, 2: 129, 3: 129, 4: 65, 5: 65, 6: 65}.get(a.block, 33)
    blk = InvertedResidual(sp)
    init_random(blk, 1)
    blk.eval()
    B = a.batch
    x = (torch.randn(B, H, H, sp.cin, device=dev)).to(torch.bfloat16)
    ew = eb = None
    if blk.expand is not None:
        ew, eb = blk.expand.fold()
        ew = ew[:, :, 0, 0]
    dwf, dbf = blk.dw.fold()
    pwf, pbf = blk.project.fold()
    P = K.pack_fused_ir(ew, eb, dwf[:, 0], dbf, pwf[:, :, 0, 0], pbf, Cin=sp.cin, hid=sp.hidden,
                        Cout=sp.cout, stride=sp.stride, residual=sp.residual, device=dev,
                        dil=sp.dilation)
    OH = (H - 1) // sp.stride + 1
    out = torch.empty(B, OH, OH, sp.cout, dtype=torch.bfloat16, device=dev)
    print(f"block {a.block}: {sp} H={H}")
    for t in a.tiles.split(","):
        ty, tx = map(int, t.split("x"))
        run = lambda: K.fused_ir(x, P, out, B=B, IH=H, IW=H, OH=OH, OW=OH, tile=(ty, tx))
        try:
            run()
        except Exception as e:  # noqa: BLE001
            print(f"  tile {t}: {e}")
            continue
        for _ in range(3):
            run()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(a.reps):
            run()
        en.record()
        torch.cuda.synchronize()
        print(f"  tile {t}: {st.elapsed_time(en) * 1e3 / a.reps:8.1f} us", flush=True)
        if a.trace:
            tr = torch.zeros(128, dtype=torch.int64, device=dev)
            K.fused_ir(x, P, out, B=B, IH=H, IW=H, OH=OH, OW=OH, tile=(ty, tx), trace=tr)
            torch.cuda.synchronize()
            v = tr.cpu().numpy()
            t0 = v[0]
            marks = [(i, int(v[i] - t0)) for i in range(128) if v[i]]
            print("    timeline (s_memtime ticks since start):", marks[:40])


if __name__ == "__main__":
    main()
