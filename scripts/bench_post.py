"""Microbenchmark of the device post-processing (postprocess.hip) at the headline
shape: B=32 label maps of 513x513 cropped to 513x385 (640x480 letterbox).

python scripts/bench_post.py [--reps 20]  -> ms per call for planted-blob maps and
for nearly uniform maps (what a random-init model produces), per SSA_QUAD_BLOCKS.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_server_amd.labels import pascal_colormap  # noqa: E402
from semantic_segmentation_server_amd.postprocess.device import DevicePostprocess  # noqa: E402
from semantic_segmentation_server_amd.postprocess.synthetic import random_label_map  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--blocks", default="64,128,256,512")
    ap.add_argument("--env", default="SSA_QUAD_BLOCKS", help="variable the --blocks values go to")
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, H, W, ch, cw = 32, 513, 513, 385, 513
    rng = np.random.default_rng(0)
    planted = np.stack([random_label_map(rng, H, W, n_blobs=8) for _ in range(B)])
    flat = np.zeros((B, H, W), np.uint8)
    flat[:, :, 200:] = 12
    post = DevicePostprocess(dev, H, W, pascal_colormap())
    for name, maps in (("planted", planted), ("flat", flat)):
        lab = torch.from_numpy(maps).to(dev)
        line = [name]
        for qb in a.blocks.split(","):
            os.environ[a.env] = qb
            for _ in range(3):
                post.run(lab, cw, ch, 0.05 * H * W)
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(a.reps):
                rec = post.run(lab, cw, ch, 0.05 * H * W)
            en.record()
            torch.cuda.synchronize()
            line.append(f"qb{qb}={st.elapsed_time(en) / a.reps * 1e3:7.1f}us(n={rec[:, 0].sum().item():.0f})")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
