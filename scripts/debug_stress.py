"""Localise the concurrency-only label mismatch (VERDICT r2 Weak #1) to one kernel.

Plan copy 0 is run once sequentially and every leaf kernel call's outputs are
snapshotted. Then, while NOISE other plan copies replay their captured graphs
back to back on their own streams (the slot-parallel situation: kernels of other
copies share the CUs), each leaf of copy 0 is re-run REPS times on its own stream
from its (unchanged) inputs and its outputs are compared on the device with the
snapshot after every run.

  mode leaf: leaf L alone, REPS times (an intra-kernel race: wave skew, LDS-DMA
             counting, missing barriers)
  mode seq : the whole leaf sequence REPS times with a compare after every leaf
             (adds kernel-boundary hand-offs under co-residence)

  python scripts/debug_stress.py B S WxH REPS NOISE MODE    e.g. 2 257 160x120 200 2 leaf
"""
import os
import sys

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.models.hip_model import Choice  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
S = int(sys.argv[2]) if len(sys.argv) > 2 else 257
cw, ch = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "160x120").split("x"))
REPS = int(sys.argv[4]) if len(sys.argv) > 4 else 200
NOISE = int(sys.argv[5]) if len(sys.argv) > 5 else 2
MODE = sys.argv[6] if len(sys.argv) > 6 else "leaf"
ONLY = os.environ.get("ONLY", "")  # comma list of leaf indices (mode leaf)

eng = Engine(C.Config(backend="hip", batch=B, input_size=S, graph=False, min_area_ratio=0.002),
             torch.device("cuda"))
eng.set_camera(cw, ch)
hm = eng._hip_model
src = SyntheticSource(cw, ch, seed=7, pool=4)
frames = [torch.from_numpy(np.ascontiguousarray(src.read_batch(B)[0])).cuda() for _ in range(2)]
ops, bufs = hm._plan(B, ch, cw)


def leaves(ol, prefix=""):
    for i, op in enumerate(ol):
        if isinstance(op, Choice):
            name, sub = op.variants[op.pick]
            yield from leaves(sub, f"{op.name}:{name}/")
        else:
            yield f"{prefix}{i}", op


LEAVES = list(leaves(ops))
ACT = {n: t for n, t in bufs.items() if isinstance(t, torch.Tensor) and t.is_cuda
       and t.dtype in (torch.bfloat16, torch.float16, torch.float32, torch.uint8)
       and not n.startswith(("pool_w", "aspp_proj_wt"))}
args = (frames[0], eng.lut_x, eng.lut_y)

# reference: zero-filled buffers, one sequential pass, per-leaf written buffers
for t in ACT.values():
    t.zero_()
torch.cuda.synchronize()
prev = {n: t.clone() for n, t in ACT.items()}
REF = []
for name, op in LEAVES:
    op(*args)
    torch.cuda.synchronize()
    cur = {n: t.clone() for n, t in ACT.items()}
    REF.append({n: cur[n] for n in ACT if not torch.equal(cur[n], prev[n])})
    prev = cur

# noise: captured graphs of plan copies 1..NOISE on their own streams
noise = []
for k in range(1, NOISE + 1):
    out = torch.empty((B, S, S), dtype=torch.uint8, device="cuda")
    hm.segment(frames[k % 2], eng.lut_x, eng.lut_y, out=out, part=k)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            hm.segment(frames[k % 2], eng.lut_x, eng.lut_y, out=out, part=k)
    noise.append((s, g))
torch.cuda.synchronize()
main = torch.cuda.Stream()
bad = torch.zeros(len(LEAVES), dtype=torch.int32, device="cuda")


def kick_noise(n):
    for s, g in noise:
        with torch.cuda.stream(s):
            for _ in range(n):
                g.replay()


DETAIL = os.environ.get("DETAIL", "0") == "1"
detail = []


def check(li):
    for n, r in REF[li].items():
        ne = (ACT[n] != r)
        bad[li] += ne.any().to(torch.int32)
        if DETAIL:  # per-buffer mismatch counts + a copy of the output, inspected on the host
            detail.append((li, n, ne.sum(), ACT[n].clone()))


print(f"B={B} S={S} {len(LEAVES)} leaves, noise copies {NOISE}, mode {MODE}, reps {REPS}", flush=True)
if MODE == "leaf":
    sel = [int(v) for v in ONLY.split(",")] if ONLY else range(len(LEAVES))
    # every leaf's inputs are in place after the reference pass (buffers are written once)
    for li in sel:
        name, op = LEAVES[li]
        done = 0
        while done < REPS:
            n = min(50, REPS - done)
            kick_noise(max(2, n // 8))
            with torch.cuda.stream(main):
                for _ in range(n):
                    op(*args)
                    check(li)
            done += n
            torch.cuda.synchronize()
        print(f"  leaf {li:2d} {name:45s} mismatching runs {int(bad[li])} / {REPS}", flush=True)
        if DETAIL:
            shown = 0
            for lj, n, cnt, val in detail:
                c = int(cnt)
                if c and shown < 6:
                    r = REF[lj][n]
                    idx = (val != r).view(-1).nonzero()[:6].view(-1).tolist()
                    fv, fr = val.view(-1).float(), r.view(-1).float()
                    print(f"      {n}: {c}/{val.numel()} differ; at {idx}: got "
                          f"{[round(fv[i].item(), 5) for i in idx]} want {[round(fr[i].item(), 5) for i in idx]}",
                          flush=True)
                    shown += 1
            detail.clear()
else:
    done = 0
    while done < REPS:
        kick_noise(4)
        with torch.cuda.stream(main):
            for li, (name, op) in enumerate(LEAVES):
                op(*args)
                check(li)
        done += 1
        if done % 10 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    for li, (name, _) in enumerate(LEAVES):
        print(f"  leaf {li:2d} {name:45s} mismatching passes {int(bad[li])} / {REPS}", flush=True)
print("total mismatches", int(bad.sum()), flush=True)
