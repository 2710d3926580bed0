"""Microbench of the config-4 MFMA stem (DeepLabv3-ResNet50: 7x7 s2 conv 3 -> 64 on the
letterboxed 2048x1024 camera frame at 1025^2, B=8, int8 out) over its tile / wave variants:
mean time per launch from HIP events. Under ``rocprofv3 --pmc`` it gives each variant's
counters (a handful of dispatches per variant).

    python scripts/bench_stem.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from semantic_segmentation_server_amd.ops import hip_ops as K  # noqa: E402
from semantic_segmentation_server_amd.ops import reference_ops as R  # noqa: E402


def main(reps: int = 20) -> int:
    B, Wc, Hc, S, k, C = 8, 2048, 1024, 1025, 7, 64
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    frames = torch.from_numpy(rng.integers(0, 256, (B, Hc, Wc, 3), dtype=np.uint8)).to(dev)
    lx, ly, *_ = R.letterbox_luts(Wc, Hc, S, S)
    lx = torch.tensor(np.array(lx), dtype=torch.int32, device=dev)
    ly = torch.tensor(np.array(ly), dtype=torch.int32, device=dev)
    g = torch.Generator().manual_seed(1)
    w = (torch.randn(k * k * 3, C, generator=g) / 8).to(dev)
    b = torch.randn(C, generator=g).to(dev)
    wpk = K.pack_stem_mfma(w, k, C)
    OH = OW = (S - 1) // 2 + 1
    out = torch.empty(B, OH, OW, C, dtype=torch.int8, device=dev)
    variants = [("mfma16x16", (16, 16), False), ("mfmaw16x16", (16, 16), True),
                ("mfmaw16x32", (16, 32), True), ("mfmaw32x32", (32, 32), True)]
    for name, tile, pw in variants:
        def run():
            K.stem_mfma(frames, lx, ly, wpk, b, out, H=S, W=S, OH=OH, OW=OW, Cout=C, k=k, stride=2,
                        act="relu", out_scale=0.05, tile=tile, per_wave=pw)
        run()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(reps):
            run()
        en.record()
        en.synchronize()
        print(f"{name:12s} {st.elapsed_time(en) / reps * 1e3:8.1f} us", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]) if len(sys.argv) > 1 else 20))
