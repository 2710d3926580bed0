"""Where the inter-step GPU idle time comes from: per-step wall time of N back-to-back
graph replays at the bench config, alone and with what the pipeline adds between
them (the D2H copy of the packed records into pinned memory, an event record)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402


def main():
    B = 32
    eng = Engine(C.Config(backend="hip", batch=B, graph=True), torch.device("cuda", 0))
    eng.set_camera(640, 480)
    from semantic_segmentation_server_amd.runtime.sources import SyntheticSource
    src = SyntheticSource(640, 480, seed=1, pool=8)
    bufs = [torch.from_numpy(src.read_batch(B)[0]).to("cuda") for _ in range(2)]
    if os.environ.get("ZERO_FRAMES") == "1":
        for b in bufs:
            b.zero_()
    eng.bind_inputs(bufs)
    _, post = eng.run_device(bufs[0])
    eng.run_device(bufs[1])
    host = torch.empty(post.shape, dtype=post.dtype).pin_memory()
    N = 30

    def timed(name, body):
        for k in range(3):
            body(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(N):
            body(k)
        torch.cuda.synchronize()
        print(f"{name:28s} {(time.perf_counter() - t0) / N * 1e6:8.1f} us/step", flush=True)

    timed("replay only (same buf)", lambda k: eng.run_device(bufs[0]))
    timed("replay only (alternating)", lambda k: eng.run_device(bufs[k % 2]))
    timed("replay + D2H", lambda k: (eng.run_device(bufs[k % 2]), host.copy_(post, non_blocking=True)))
    timed("replay + event", lambda k: (eng.run_device(bufs[k % 2]), torch.cuda.Event().record()))

    def full(k):
        eng.run_device(bufs[k % 2])
        host.copy_(post, non_blocking=True)
        torch.cuda.Event().record()
    timed("replay + D2H + event", full)
    dd = torch.empty(post.shape, dtype=post.dtype, device="cuda")
    timed("replay + D2D", lambda k: (eng.run_device(bufs[k % 2]), dd.copy_(post, non_blocking=True)))


if __name__ == "__main__":
    main()
