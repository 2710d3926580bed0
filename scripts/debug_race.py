"""Bisect a concurrency-only mismatch: run plan copies (parts 0..2) of the HIP model on three
streams at once and compare with sequential results, with every Choice whose name matches
FORCE (comma list of name-prefix=variant) pinned to that variant.
  python scripts/debug_race.py REPS "block=unfused,aspp.branches=separate" """
import os
import sys

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
import test_hip_kernels as T  # noqa: E402
from semantic_segmentation_server_amd.models.hip_model import Choice  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
force = [kv.split("=") for kv in sys.argv[2].split(",")] if len(sys.argv) > 2 and sys.argv[2] else []
B = int(os.environ.get("RACE_B", "2"))
S = int(os.environ.get("RACE_S", "257"))
CW, CH = (int(v) for v in os.environ.get("RACE_CAM", "160x120").split("x"))
eng = Engine(T._small_cfg(graph=True, batch=B, input_size=S, min_area_ratio=0.002), torch.device("cuda"))
src = SyntheticSource(CW, CH, seed=7, pool=4)
eng.set_camera(CW, CH)
hm = eng._hip_model
fr = [torch.from_numpy(np.ascontiguousarray(src.read_batch(B)[0])).cuda() for _ in range(3)]
for part in range(3):
    hm.segment(fr[0], eng.lut_x, eng.lut_y, part=part)


def pin(ops):
    for op in ops:
        if isinstance(op, Choice):
            for pre, var in force:
                if op.name == pre or (pre.endswith("*") and op.name.startswith(pre[:-1])):
                    idx = [n for n, _ in op.variants]
                    if var in idx:
                        op.pick = idx.index(var)
            for _, v in op.variants:
                pin(v)


picks = []
for part in range(3):
    ops = hm._plan(B, CH, CW, part)[0]
    pin(ops)
    picks.append({op.name: op.variants[op.pick][0] for op in ops if isinstance(op, Choice)})
assert picks[0] == picks[1] == picks[2]
print("picks:", picks[0], flush=True)
ref = {}
for i, f in enumerate(fr):
    ref[i] = hm.segment(f, eng.lut_x, eng.lut_y, part=0).clone()
torch.cuda.synchronize()
ss = [torch.cuda.Stream() for _ in range(3)]
labs = [torch.empty_like(ref[0]) for _ in range(3)]
bad = 0
for rep in range(reps):
    for part in range(3):
        with torch.cuda.stream(ss[part]):
            hm.segment(fr[(rep + part) % 3], eng.lut_x, eng.lut_y, out=labs[part], part=part)
    torch.cuda.synchronize()
    for part in range(3):
        d = (labs[part] != ref[(rep + part) % 3]).sum().item()
        bad += d > 0
print(f"FORCE={sys.argv[2] if len(sys.argv) > 2 else ''}: concurrent mismatching runs {bad} / {3 * reps}", flush=True)
