"""Which plan variant makes label maps depend on history? (tests/test_hip_kernels.py::
test_plan_is_a_function_of_the_frame, per variant.)

For the 257^2 / 160x120 B=2 plan: every Choice is switched through its variants (others at
the autotuned picks); per variant the frame-0 labels are compared across (a) a second run
after another frame, (b) a run after the plan's float/bf16/uint8 buffers were NaN-filled.
Prints the variants whose labels differ.

    python scripts/debug_history.py [only-substring]
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.models.hip_model import Choice  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402


def main() -> None:
    only = sys.argv[1] if len(sys.argv) > 1 else ""
    dev = torch.device("cuda", 0)
    B, S, cam = 2, 257, (160, 120)
    eng = Engine(C.Config(input_size=S, batch=B, backend="hip", graph=True, min_area_ratio=0.002), dev)
    src = SyntheticSource(cam[0], cam[1], seed=7, pool=4)
    eng.set_camera(*cam)
    fr = [torch.from_numpy(np.ascontiguousarray(src.read_batch(B)[0])).to(dev) for _ in range(3)]
    hm = eng._hip_model
    hm.segment(fr[0], eng.lut_x, eng.lut_y)
    print("picks:", hm.choices, flush=True)
    ops, bufs = hm._plan(B, cam[1], cam[0])

    def poison():
        for n, t in bufs.items():
            if not isinstance(t, torch.Tensor) or not t.is_cuda or n.startswith(("pool_w", "aspp_proj_wt", "const_")):
                continue
            if t.dtype == torch.uint8:
                t.fill_(0xC0)
            elif t.dtype == torch.float32:
                t.view(torch.int32).fill_(0x7FC07FC0)
            elif t.dtype in (torch.bfloat16, torch.float16):
                t.view(torch.int16).fill_(0x7FC0)

    def check() -> str:
        a0 = hm.segment(fr[0], eng.lut_x, eng.lut_y).clone()
        hm.segment(fr[1], eng.lut_x, eng.lut_y)
        a1 = hm.segment(fr[0], eng.lut_x, eng.lut_y).clone()
        poison()
        a2 = hm.segment(fr[0], eng.lut_x, eng.lut_y).clone()
        torch.cuda.synchronize()
        return ("ok" if torch.equal(a0, a1) else "HIST") + "/" + ("ok" if torch.equal(a0, a2) else "POISON")

    print("committed:", check(), flush=True)
    choices = [o for o in ops if isinstance(o, Choice)]
    nested = [o for c in choices for _, vops in c.variants for o in vops if isinstance(o, Choice)]
    for op in choices + nested:
        if only and only not in op.name:
            continue
        keep = op.pick
        bad = []
        for i, (name, _) in enumerate(op.variants):
            op.pick = i
            try:
                r = check()
            except Exception as ex:  # noqa: BLE001
                r = f"ERR({type(ex).__name__})"
            if r != "ok/ok":
                bad.append(f"{name}={r}")
        op.pick = keep
        check()
        print(f"{op.name}: {len(op.variants)} variants, bad: {bad}", flush=True)


if __name__ == "__main__":
    main()
