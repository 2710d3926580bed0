"""Find a kernel that writes outside its buffers: every plan buffer gets 0x5A guard bands
(SSA_GUARD_BYTES), the plan's ops run one at a time (every Choice variant too) and the
bands are checked after each launch."""
import os
import sys

os.environ.setdefault("SSA_GUARD_BYTES", "65536")
import numpy as np  # noqa: E402
import torch  # noqa: E402

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
import test_hip_kernels as T  # noqa: E402
from semantic_segmentation_server_amd.models.hip_model import Choice  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
size = int(sys.argv[2]) if len(sys.argv) > 2 else 257
eng = Engine(T._small_cfg(graph=True, batch=B, input_size=size, min_area_ratio=0.002), torch.device("cuda"))
cam = (160, 120) if size < 513 else (640, 480)
src = SyntheticSource(*cam, seed=7, pool=4)
eng.set_camera(*cam)
hm = eng._hip_model
f = torch.from_numpy(np.ascontiguousarray(src.read_batch(B)[0])).cuda()
hm._guards.clear()
ops, bufs = hm._plan(B, cam[1], cam[0], part=5)


def check(tag):
    torch.cuda.synchronize()
    bad = []
    for name, raw, g, nb in hm._guards:
        lo = raw[:g]
        hi = raw[g + nb:]
        if (lo != 0x5A).any() or (hi != 0x5A).any():
            nlo = int((lo != 0x5A).sum())
            nhi = int((hi != 0x5A).sum())
            bad.append(f"{name}(before {nlo} B, after {nhi} B)")
            lo.fill_(0x5A)
            hi.fill_(0x5A)
    if bad:
        print(f"GUARD HIT after {tag}: {', '.join(bad)}", flush=True)


check("plan build")
args = (f, eng.lut_x, eng.lut_y)


def run(op, tag):
    if isinstance(op, Choice):
        for name, vops in op.variants:
            for j, o in enumerate(vops):
                run(o, f"{tag}/{op.name}:{name}[{j}]")
    else:
        op(*args)
        check(tag)


for i, op in enumerate(ops):
    run(op, f"op{i}")
print("guard scan done", len(hm._guards), "buffers", flush=True)
