"""World-size-1 rehearsal of the multi-GPU data path on one GPU:
a real RCCL process group (SSA_FORCE_PG=1, backend nccl) with the gloo control group,
the DP pipeline with the RCCL record gather (one [records | metadata] collective to
rank 0, then the pinned-host write kernel), lag 2 on slot-parallel plan copies; the
records must equal an eager synchronous engine's on the same frames. ``scatter`` as the
first argument: rank 0 uploads the node batch and RCCL-scatters it on the slot streams
(X1, VERDICT r3 #3d). Prints 'OK gather=<mode> pg=<backend> records=<n>'
(tests/test_hip_kernels.py runs it in a child process so the process group does not
outlive it)."""
import os
import sys

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
os.environ.setdefault("SSA_FORCE_PG", "1")
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.parallel import dist as D  # noqa: E402
from semantic_segmentation_server_amd.parallel.dp import DataParallelPipeline  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.results import ResultHub  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

ctx = D.init("nccl")
assert ctx.backend == "nccl" and ctx.cpu_group is not None, ctx
eng = Engine(C.Config(backend="hip", batch=2, input_size=257, graph=True, min_area_ratio=0.002),
             ctx.device)
src = SyntheticSource(160, 120, seed=7, pool=4)
batches = [torch.from_numpy(np.ascontiguousarray(src.read_batch(2)[0])) for _ in range(2)]
eng.set_camera(160, 120)
want = []
for k in range(6):
    _, post = eng._step_device(batches[k % 2].to(ctx.device))
    r = eng._hip_post.fetch(post, [k * 2, k * 2 + 1], [0.0, 0.0], [0, 0], eng.W, eng.H)
    want.extend(zip(r["frame"].tolist(), r["label"].tolist(), r["area"].round(6).tolist()))
torch.cuda.synchronize()
hub = ResultHub(1)
ingest = sys.argv[1] if len(sys.argv) > 1 else "local"
pipe = DataParallelPipeline(ctx, eng, 160, 120, 2, ingest, hub, lag=1, gather="rccl")  # auto: lag 2
assert pipe.lag == 2 and eng.slot_parallel, (pipe.lag, eng.slot_parallel)
got = []
pipe.prefetch(batches[0].pin_memory())
for k in range(6):
    recs = pipe.step(next_frames=batches[(k + 1) % 2].pin_memory() if k < 5 else None)
    got.extend(zip(recs["frame"].tolist(), recs["label"].tolist(), recs["area"].round(6).tolist()))
last = pipe.flush()
got.extend(zip(last["frame"].tolist(), last["label"].tolist(), last["area"].round(6).tolist()))
torch.cuda.synchronize()
assert len(want) > 0
assert sorted(got) == sorted(want), (len(got), len(want))
assert hub.depth == len(want)
D.barrier(ctx)
assert pipe.frame_order_errors == 0 and sum(pipe.stream_frames.values()) == 12
print(f"OK ingest={ingest} gather={pipe.gather_mode} pg={ctx.backend} lag={pipe.lag} records={len(got)}",
      flush=True)
D.destroy(ctx)
