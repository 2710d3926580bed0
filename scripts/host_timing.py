"""Host-side time per pipeline stage at the bench config (where the GPU waits on
the host between steps): wall time of graph replay, H2D prefetch enqueue, record
collection and the whole step, per step, after warmup.

python scripts/host_timing.py [--steps 30] [--lag 1]"""
import argparse
import os
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--lag", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    ctx = D.init()
    cfg = C.Config(backend="hip", batch=a.batch, graph=True)
    eng = Engine(cfg, ctx.device)
    hub = ResultHub(1, maxlen=4096)
    pipe = DataParallelPipeline(ctx, eng, 640, 480, a.batch, "local", hub, 1, lag=a.lag)
    src = SyntheticSource(640, 480, seed=1, pool=8)
    hb = [torch.from_numpy(np.ascontiguousarray(src.read_batch(a.batch)[0])).pin_memory() for _ in range(2)]
    T = {}

    def wrap(obj, name):
        f = getattr(obj, name)

        def g(*args, **kw):
            t0 = time.perf_counter()
            r = f(*args, **kw)
            T.setdefault(name, []).append(time.perf_counter() - t0)
            return r
        setattr(obj, name, g)
    wrap(eng, "run_device")
    wrap(pipe, "prefetch")
    wrap(pipe, "_collect")
    pipe.prefetch(hb[0])
    steps = []
    for k in range(a.steps):
        t0 = time.perf_counter()
        pipe.step(next_frames=hb[(k + 1) % 2])
        steps.append(time.perf_counter() - t0)
    pipe.flush()
    torch.cuda.synchronize()
    w = a.steps // 3
    for n, v in [("step", steps)] + sorted(T.items()):
        v = np.array(v[w:]) * 1e6
        print(f"{n:12s} median {np.median(v):8.1f} us  max {v.max():8.1f}  n={len(v)}")


if __name__ == "__main__":
    main()
