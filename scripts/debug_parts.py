"""Do plan copies (parts) of the HIP model produce bit-identical label maps? Runs the same
frames through parts 0/1/2 (sequentially, then concurrently on three streams) and compares."""
import os
import sys

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
import test_hip_kernels as T  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

eng = Engine(T._small_cfg(graph=True, batch=2, input_size=257, min_area_ratio=0.002), torch.device("cuda"))
src = SyntheticSource(160, 120, seed=7, pool=4)
eng.set_camera(160, 120)
hm = eng._hip_model
fr = [torch.from_numpy(np.ascontiguousarray(src.read_batch(2)[0])).cuda() for _ in range(3)]
outs = {}
for part in (0, 1, 2):
    for i, f in enumerate(fr):
        outs[(part, i)] = hm.segment(f, eng.lut_x, eng.lut_y, part=part).clone()
torch.cuda.synchronize()
for i in range(3):
    for part in (1, 2):
        d = (outs[(part, i)] != outs[(0, i)]).sum().item()
        print(f"sequential frame-batch {i} part {part} vs 0: {d} differing pixels", flush=True)
# concurrent: three parts on three streams, repeated
ss = [torch.cuda.Stream() for _ in range(3)]
labs = [torch.empty_like(outs[(0, 0)]) for _ in range(3)]
bad = 0
for rep in range(20):
    for part in range(3):
        with torch.cuda.stream(ss[part]):
            hm.segment(fr[(rep + part) % 3], eng.lut_x, eng.lut_y, out=labs[part], part=part)
    torch.cuda.synchronize()
    for part in range(3):
        d = (labs[part] != outs[(0, (rep + part) % 3)]).sum().item()
        bad += d > 0
        if d:
            print(f"concurrent rep {rep} part {part}: {d} differing pixels", flush=True)
print("concurrent mismatching runs:", bad, flush=True)
