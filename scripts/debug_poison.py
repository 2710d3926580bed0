"""Find kernels whose output depends on state they did not write (VERDICT r2 Weak #1).

Runs the HIP plan one leaf kernel call at a time, four ways, from the same frames:

  A  every plan activation buffer zero-filled first            (reference, snapshots)
  B  every plan activation buffer NaN-filled first (0x7FC0 / 0xC0 for uint8)
  C  zero-filled, and before EVERY leaf every CU's LDS and every SIMD's register file
     NaN-poisoned (ops.hip_ops.poison_chip)
  D  same as A again (sequential determinism)

For each leaf L, the buffers L wrote in run A (changed from the previous leaf) are
compared with run A: a difference in B means L read global bytes nobody wrote (or
does not write all of its output); in C, L read LDS / registers it did not set; in D,
L is not deterministic. The first leaf that differs names the kernel.

  python scripts/debug_poison.py B S [cam WxH] [runs]   e.g.  2 257 160x120 ABCD
"""
import os
import sys

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.models.hip_model import Choice  # noqa: E402
from semantic_segmentation_server_amd.ops import hip_ops as K  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
S = int(sys.argv[2]) if len(sys.argv) > 2 else 257
cw, ch = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "160x120").split("x"))
runs = sys.argv[4] if len(sys.argv) > 4 else "ABCD"
force = os.environ.get("FORCE", "")  # "name=variant,..." pins, as scripts/debug_race.py

eng = Engine(C.Config(backend="hip", batch=B, input_size=S, graph=False, min_area_ratio=0.002),
             torch.device("cuda"))
eng.set_camera(cw, ch)
hm = eng._hip_model
src = SyntheticSource(cw, ch, seed=7, pool=4)
frames = torch.from_numpy(np.ascontiguousarray(src.read_batch(B)[0])).cuda()
args = (frames, eng.lut_x, eng.lut_y)
ops, bufs = hm._plan(B, ch, cw)
if force:
    pins = [kv.split("=") for kv in force.split(",")]

    def pin(ol):
        for op in ol:
            if isinstance(op, Choice):
                for pre, var in pins:
                    if op.name == pre or (pre.endswith("*") and op.name.startswith(pre[:-1])):
                        names = [n for n, _ in op.variants]
                        if var in names:
                            op.pick = names.index(var)
                for _, v in op.variants:
                    pin(v)
    pin(ops)


def leaves(ol, prefix=""):
    for i, op in enumerate(ol):
        if isinstance(op, Choice):
            name, sub = op.variants[op.pick]
            yield from leaves(sub, f"{op.name}:{name}/")
        else:
            yield f"{prefix}{i}", op


LEAVES = list(leaves(ops))
# activation buffers only: int tables (tile orders, permutations) and packed weights are
# read-only plan constants, and poisoning an index table would fault the GPU
ACT = {n: t for n, t in bufs.items() if isinstance(t, torch.Tensor) and t.is_cuda
       and t.dtype in (torch.bfloat16, torch.float16, torch.float32, torch.uint8)
       and not n.startswith(("pool_w", "aspp_proj_wt"))}
print(f"B={B} S={S} cam={cw}x{ch}: {len(LEAVES)} leaf calls, {len(ACT)} activation buffers "
      f"({sum(t.numel() * t.element_size() for t in ACT.values()) / 2**20:.1f} MiB)", flush=True)
print("picks:", {op.name: op.variants[op.pick][0] for op in ops if isinstance(op, Choice)}, flush=True)


def fill(nan: bool):
    for t in ACT.values():
        if not nan:
            t.zero_()
        elif t.dtype == torch.uint8:
            t.fill_(0xC0)
        elif t.dtype == torch.float32:
            t.view(torch.int32).fill_(0x7FC07FC0)
        else:
            t.view(torch.int16).fill_(0x7FC0)


def run(init_nan: bool, chip: bool, snaps=None):
    """Returns per-leaf snapshots (when snaps is None) or per-leaf differences vs snaps."""
    fill(init_nan)
    torch.cuda.synchronize()
    out, diffs, prev = [], [], {n: t.clone() for n, t in ACT.items()}
    for li, (name, op) in enumerate(LEAVES):
        if chip:
            K.poison_chip()
        op(*args)
        torch.cuda.synchronize()
        if snaps is None:
            cur = {n: t.clone() for n, t in ACT.items()}
            wrote = [n for n in ACT if not torch.equal(cur[n], prev[n])]
            out.append((cur, wrote))
            prev = cur
        else:
            ref, wrote = snaps[li]
            d = []
            for n in wrote:
                a, b = ref[n].view(-1), ACT[n].view(-1)
                if a.dtype != torch.uint8:
                    a, b = a.view(torch.int16 if a.element_size() == 2 else torch.int32), \
                        b.view(torch.int16 if b.element_size() == 2 else torch.int32)
                nd = int((a != b).sum())
                if nd:
                    d.append((n, nd, a.numel()))
            diffs.append(d)
    return out if snaps is None else diffs


snaps = run(False, False)
for li, ((name, _), (_, wrote)) in enumerate(zip(LEAVES, snaps)):
    print(f"  leaf {li:2d} {name:45s} writes {wrote}")
labels_ref = bufs["labels"].clone()
for r in runs:
    if r == "A":
        continue
    init_nan, chip = {"B": (True, False), "C": (False, True), "D": (False, False)}[r]
    diffs = run(init_nan, chip, snaps)
    nbad = (bufs["labels"] != labels_ref).sum().item()
    first = next((li for li, d in enumerate(diffs) if d), None)
    print(f"run {r} (init {'NaN' if init_nan else 'zero'}, chip poison {chip}): label pixels "
          f"differing {nbad}; first differing leaf: "
          f"{'none' if first is None else f'{first} {LEAVES[first][0]}'}", flush=True)
    for li, d in enumerate(diffs):
        if d:
            print(f"    leaf {li:2d} {LEAVES[li][0]:45s} " +
                  ", ".join(f"{n} {nd}/{tot}" for n, nd, tot in d), flush=True)
