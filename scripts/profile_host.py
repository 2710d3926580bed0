"""Where the host thread spends a pipeline step (bench.py's loop at a given batch), by
Python function: cProfile over the timed steps of the same DataParallelPipeline the bench
drives (world size 1, HIP engine, hipGraph, lag 2). At batch 1 the host is on the critical
path (bench.py host_ms_per_step: busy ~0.10-0.13 ms of a ~0.17 ms step).

  python scripts/profile_host.py [batch] [steps]
"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.parallel import dist as D  # noqa: E402
from semantic_segmentation_server_amd.parallel.dp import DataParallelPipeline  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.results import ResultHub  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    ctx = D.init(None, device="cuda")
    cfg = C.Config(batch=B, backend="hip", graph=True)
    eng = Engine(cfg, ctx.device)
    hub = ResultHub(1, maxlen=4096)
    src = SyntheticSource(640, 480, stream=0, seed=1, pool=max(2, min(B, 8)))
    hb = [torch.from_numpy(np.ascontiguousarray(src.read_batch(B)[0])).pin_memory() for _ in range(2)]
    pipe = DataParallelPipeline(ctx, eng, 640, 480, B, "local", hub, 1, lag=2, auto_lag=False)
    pipe.prefetch(hb[0])
    for k in range(200):
        pipe.step(next_frames=hb[(k + 1) % 2])
    torch.cuda.synchronize()
    prof = cProfile.Profile()
    t0 = time.perf_counter()
    prof.enable()
    for k in range(steps):
        pipe.step(next_frames=hb[(k + 1) % 2])
    prof.disable()
    pipe.flush()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"batch {B}: {steps} steps, {dt / steps * 1e3:.4f} ms/step under cProfile")
    st = pstats.Stats(prof)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
