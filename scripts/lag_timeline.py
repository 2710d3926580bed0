"""Per-step timeline of the bench loop (why short timed windows lose throughput at lag 2).

Builds the pipeline exactly as bench.py does, runs W warmup steps + flush, then K timed
steps, and prints for every timed step the host time at which step() returned plus the
GPU start / end of that step's model graph (events on its slot stream).

  python scripts/lag_timeline.py LAG W K
"""
import os
import sys
import time

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.parallel import dist as D  # noqa: E402
from semantic_segmentation_server_amd.parallel.dp import DataParallelPipeline  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

LAG = int(sys.argv[1]) if len(sys.argv) > 1 else 2
W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
B = int(os.environ.get("TL_B", "32"))
ctx = D.init("gloo", device="cuda")
cfg = C.Config(backend="hip", batch=B, input_size=513, graph=True)
eng = Engine(cfg, ctx.device)
src = SyntheticSource(640, 480, seed=1, pool=8)
hb = [torch.from_numpy(np.ascontiguousarray(src.read_batch(B)[0])).pin_memory() for _ in range(2)]
pipe = DataParallelPipeline(ctx, eng, 640, 480, B, "local", None, lag=LAG, auto_lag=False)

# instrument the slot-parallel model replays: an event pair around each graph replay
marks = []
orig = eng.run_device


def run_device(frames):
    i = eng._slot_of.get(frames.data_ptr())
    st = eng.slot_streams[i] if getattr(eng, "slot_parallel", False) and i is not None else \
        torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    out = orig(frames)
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(st)
    marks.append((e0, e1))
    return out


eng.run_device = run_device

# host time spent in the pipeline's phases (which call blocks in a stalled step)
phase_t = []


def timed(obj, name):
    f = getattr(obj, name)

    def w(*a, **k):
        t = time.perf_counter()
        r = f(*a, **k)
        phase_t.append((name, t, time.perf_counter()))
        return r
    setattr(obj, name, w)


for nm in ("_collect", "prefetch", "_frames_for_step"):
    timed(pipe, nm)
timed(eng, "run_device")


def run(n, k0=0):
    pipe.prefetch(hb[k0 % 2])
    hs = []
    for k in range(n):
        pipe.step(next_frames=hb[(k0 + k + 1) % 2])
        hs.append(time.perf_counter())
    pipe.flush()
    return hs


import gc  # noqa: E402

gcs = []
gc.callbacks.append(lambda phase, info: gcs.append((phase, info["generation"], time.perf_counter())))
run(W)
torch.cuda.synchronize()
if os.environ.get("TL_FREEZE", "0") == "1":
    gc.collect()
    gc.freeze()
marks.clear()
gcs.clear()
phase_t.clear()
base = torch.cuda.Event(enable_timing=True)
base.record()
t0 = time.perf_counter()
if os.environ.get("TL_PROFILE", "0") == "1":
    import cProfile
    import pstats
    prof = cProfile.Profile()
    prof.enable()
    hs = run(K, W)
    prof.disable()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    pstats.Stats(prof).sort_stats("tottime").print_stats(12)
else:
    hs = run(K, W)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
print(f"lag {LAG} warmup {W} steps {K}: {K * B / (t1 - t0):.0f} frames/s, {(t1 - t0) / K * 1e3:.3f} ms/step",
      flush=True)
ev = {}
for phase, gen, t in gcs:
    ev.setdefault(gen, []).append((phase, 1e3 * (t - t0)))
for gen, lst in sorted(ev.items()):
    starts = [t for p, t in lst if p == "start"]
    stops = [t for p, t in lst if p == "stop"]
    durs = [b - a for a, b in zip(starts, stops)]
    print(f"  gc gen {gen}: {len(starts)} collections in the window, longest {max(durs or [0]):.3f} ms "
          f"at {[round(a, 2) for a, d in zip(starts, durs) if d > 0.5]}", flush=True)
slow = [(n, 1e3 * (a - t0), 1e3 * (b - a)) for n, a, b in phase_t if b - a > 5e-4]
print("  host phases > 0.5 ms:", [(n, round(a, 2), round(d, 2)) for n, a, d in slow], flush=True)
for k, ((e0, e1), h) in enumerate(zip(marks, hs)):
    print(f"  step {k:3d}: host return {1e3 * (h - t0):8.3f} ms  gpu model {base.elapsed_time(e0):8.3f} -> "
          f"{base.elapsed_time(e1):8.3f} ms ({e0.elapsed_time(e1):6.3f})", flush=True)
