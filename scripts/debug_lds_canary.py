"""Which kernel writes LDS it does not own? (the aspp_pool mismatch of
scripts/debug_pool.py: its LDS reduction state changes under plan-copy noise while its
global inputs stay correct). LDS canary workgroups (debug_poison.hip) hold a pattern in
their LDS while ONE leaf kernel call of the plan runs REPS times beside them on another
stream; a changed canary word names that leaf.

  python scripts/debug_lds_canary.py B S WxH REPS"""
import os
import sys

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.models.hip_model import Choice  # noqa: E402
from semantic_segmentation_server_amd.ops.native import hip_debug as H  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
S = int(sys.argv[2]) if len(sys.argv) > 2 else 257
cw, ch = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "160x120").split("x"))
REPS = int(sys.argv[4]) if len(sys.argv) > 4 else 50
eng = Engine(C.Config(backend="hip", batch=B, input_size=S, graph=False, min_area_ratio=0.002),
             torch.device("cuda"))
eng.set_camera(cw, ch)
hm = eng._hip_model
src = SyntheticSource(cw, ch, seed=7, pool=4)
frames = torch.from_numpy(np.ascontiguousarray(src.read_batch(B)[0])).cuda()
ops, bufs = hm._plan(B, ch, cw)
args = (frames, eng.lut_x, eng.lut_y)
hm.segment(*args)
torch.cuda.synchronize()


def leaves(ol, prefix=""):
    for i, op in enumerate(ol):
        if isinstance(op, Choice):
            name, sub = op.variants[op.pick]
            yield from leaves(sub, f"{op.name}:{name}/")
        else:
            yield f"{prefix}{i}", op


LEAVES = list(leaves(ops))
ALL = os.environ.get("ALL_VARIANTS", "0") == "1"
if ALL:  # every variant of every choice, not only the picked ones
    LEAVES = []

    def allv(ol, prefix=""):
        for i, op in enumerate(ol):
            if isinstance(op, Choice):
                for name, sub in op.variants:
                    allv(sub, f"{op.name}:{name}/")
            else:
                LEAVES.append((f"{prefix}{i}", op))
    allv(ops)
bad = torch.zeros(1, dtype=torch.int32, device="cuda")
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
print(f"B={B} S={S}: {len(LEAVES)} leaves, {REPS} reps each beside 512 canary workgroups", flush=True)
# control: canaries alone
with torch.cuda.stream(sa):
    H().lds_canary(4000, bad.data_ptr(), 512, sa.cuda_stream)
torch.cuda.synchronize()
print(f"  control (canaries alone): {int(bad)} corrupted words", flush=True)
for li, (name, op) in enumerate(LEAVES):
    bad.zero_()
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        H().lds_canary(6000, bad.data_ptr(), 512, sa.cuda_stream)
    with torch.cuda.stream(sb):
        for _ in range(REPS):
            op(*args)
    torch.cuda.synchronize()
    n = int(bad)
    print(f"  leaf {li:3d} {name:50s} corrupted canary words {n}{'   <-----' if n else ''}", flush=True)
