"""Marginal time of each device post-processing stage on the label maps the bench
really produces (random-init DeepLabv3-MNv2 on synthetic camera frames, B=32):
the pipeline is timed with SSA_POST_STAGES = 1..n (stage k's cost = t(k) - t(k-1)).
Extra env assignments on the command line (NAME=value) are applied first."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.postprocess.device import DevicePostprocess  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

NAMES = ["zero+ccl_local", "ccl_edges", "ccl_merge", "ccl_boundary", "compress", "roots", "quads",
         "tree", "select", "hist", "finalize"]


def main():
    for kv in sys.argv[1:]:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    B = 32
    eng = Engine(C.Config(backend="hip", batch=B, graph=False), torch.device("cuda", 0))
    eng.set_camera(640, 480)
    src = SyntheticSource(640, 480, seed=1, pool=8)
    frames = torch.from_numpy(src.read_batch(B)[0]).cuda()
    labels, _ = eng._step_device(frames)
    labels = labels.clone()
    post = DevicePostprocess(eng.device, eng.H, eng.W, eng.palette, eng.cfg.max_segments)
    prev = 0.0
    for k in range(1, len(NAMES) + 1):
        os.environ["SSA_POST_STAGES"] = str(k)
        for _ in range(3):
            post.run(labels, eng.crop_w, eng.crop_h, eng.min_area)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(20):
            post.run(labels, eng.crop_w, eng.crop_h, eng.min_area)
        en.record()
        torch.cuda.synchronize()
        t = st.elapsed_time(en) / 20 * 1e3
        print(f"{NAMES[k - 1]:16s} {t - prev:7.1f} us   (cumulative {t:7.1f})", flush=True)
        prev = t


if __name__ == "__main__":
    main()
