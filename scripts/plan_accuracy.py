"""Per-variant accuracy of a committed plan at the headline shape (513^2, 640x480 camera).

For batch B, every plan step (Choice, nested ones included) is switched through each of
its variants with all other steps at the committed picks; the logits are compared with
the fp32 torch model (relative error and argmax agreement after the bilinear upsample).
Finds the kernel variant behind an accuracy gap of a plan
(tests/test_hip_kernels.py::test_hip_model_headline_shape_matches_torch).

    python scripts/plan_accuracy.py [B] [only-substring] [engine]

``engine``: the smoke()'s setup instead -- the serving Engine's model (BN calibrated on
the calibration frames) and SyntheticSource frames with planted regions.
"""
from __future__ import annotations

import copy
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.models.deeplab import build_model  # noqa: E402
from semantic_segmentation_server_amd.models.hip_model import Choice, HipDeepLab  # noqa: E402
from semantic_segmentation_server_amd.ops import reference_ops as R  # noqa: E402


def main() -> None:
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    only = sys.argv[2] if len(sys.argv) > 2 else ""
    dev = torch.device("cuda", 0)
    S = 513
    lx, ly, *_ = R.letterbox_luts(640, 480, S, S)
    if len(sys.argv) > 3 and sys.argv[3] == "engine":
        from semantic_segmentation_server_amd.runtime.engine import Engine
        from semantic_segmentation_server_amd.runtime.sources import SyntheticSource
        eng = Engine(C.Config(backend="hip", batch=B, input_size=S, graph=False), dev)
        model, hm = eng.model, eng._hip_model
        fr, _, _ = SyntheticSource(640, 480, seed=7, pool=4).read_batch(B)
        frames = torch.from_numpy(np.ascontiguousarray(fr))
    else:
        model = build_model("mnv2", 21, calibrate_hw=129)
        hm = HipDeepLab(model, dev, C.Config(input_size=S, batch=B, backend="hip", graph=False))
        rng = np.random.default_rng(9)
        frames = torch.from_numpy(rng.integers(0, 256, (B, 480, 640, 3), dtype=np.uint8))
    x = R.preprocess(frames, lx, ly).to(dev)
    with torch.no_grad():
        ref = copy.deepcopy(model).to(dev)(x).float()
        bf = copy.deepcopy(model).to(dev, torch.bfloat16)(x.to(torch.bfloat16)).float()
    ref_lab = R.upsample_argmax(ref.cpu(), S, S)
    fd, tx, ty = frames.to(dev), torch.tensor(lx, device=dev), torch.tensor(ly, device=dev)

    def score(lg: torch.Tensor):
        got = lg.float().permute(0, 3, 1, 2)
        e = ((got - ref).norm() / ref.norm()).item()
        a = (R.upsample_argmax(got.cpu(), S, S) == ref_lab).float().mean().item()
        return e, a

    e_bf, a_bf = score(bf.permute(0, 2, 3, 1))
    print(f"B={B} torch-bf16: rel {e_bf:.4f} agree {a_bf:.4f}")
    base = score(hm.logits(fd, tx, ty).clone())
    print(f"B={B} committed plan: rel {base[0]:.4f} agree {base[1]:.4f}", flush=True)
    ops = hm._plan(B, 480, 640)[0]
    choices = [o for o in ops if isinstance(o, Choice)]
    nested = [o for c in choices for _, vops in c.variants for o in vops if isinstance(o, Choice)]
    for op in choices + nested:
        if only and only not in op.name:
            continue
        keep = op.pick
        rows = []
        for i, (name, _) in enumerate(op.variants):
            op.pick = i
            try:
                e, a = score(hm.logits(fd, tx, ty).clone())
                rows.append(f"{name}{'*' if i == keep else ''}={e:.4f}/{a:.4f}")
            except Exception as ex:  # noqa: BLE001 - a variant that refuses this shape
                rows.append(f"{name}=ERR({type(ex).__name__})")
        op.pick = keep
        torch.cuda.synchronize()
        print(f"{op.name}: " + " ".join(rows), flush=True)


if __name__ == "__main__":
    main()
