"""Which stage of the ASPP image-pooling op goes wrong under plan-copy noise
(scripts/debug_stress.py found leaf aspp_pool). Per run, aspp_pool_kernel dumps the
GAP means it reduced (s_gap) and the pooled vector (s_pool); both are compared with
values recomputed on the host from the (correct) partial sums.

  python scripts/debug_pool.py REPS MODE     MODE bit0: agent acquire fence at kernel
  start; bit1: skip gap_partial (reuse ws)"""
import os
import sys

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.ops.native import hip as H  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 400
MODE = int(sys.argv[2]) if len(sys.argv) > 2 else 0
B, S, cw, ch = 2, 257, 160, 120
eng = Engine(C.Config(backend="hip", batch=B, input_size=S, graph=False, min_area_ratio=0.002),
             torch.device("cuda"))
eng.set_camera(cw, ch)
hm = eng._hip_model
src = SyntheticSource(cw, ch, seed=7, pool=4)
frames = [torch.from_numpy(np.ascontiguousarray(src.read_batch(B)[0])).cuda() for _ in range(2)]
ops, bufs = hm._plan(B, ch, cw)
hm.segment(frames[0], eng.lut_x, eng.lut_y)
torch.cuda.synchronize()
x = bufs["b16_out"]
ws, ib = bufs["gap_ws"], bufs["img_bias"]
w1t, w2t, b1 = bufs["pool_w1t"], bufs["pool_w2t"], hm.pool_b
Bq, h, w, Cc = x.shape
N = ib.shape[1]
ib_ref = ib.clone()
ws_ref = ws.clone()
part = ws_ref.view(B, 16, Cc).double().sum(1) / (h * w)
pool_ref = torch.relu(part @ w1t.double() + b1.double())
noise = []
for k in (1, 2):
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
dbg = torch.zeros((REPS, B, Cc + N), dtype=torch.float32, device="cuda")
outs = torch.zeros((REPS, B, N), dtype=torch.float32, device="cuda")
wss = torch.zeros((REPS,) + tuple(ws.shape), dtype=torch.float32, device="cuda")
done = 0
while done < REPS:
    n = min(50, REPS - done)
    for s, g in noise:
        with torch.cuda.stream(s):
            for _ in range(max(2, n // 8)):
                g.replay()
    with torch.cuda.stream(main):
        for r in range(done, done + n):
            H().aspp_pool(x.data_ptr(), ws.data_ptr(), w1t.data_ptr(), b1.data_ptr(), w2t.data_ptr(),
                          ib.data_ptr(), B, h * w, Cc, N, main.cuda_stream, dbg[r].data_ptr(), MODE)
            outs[r].copy_(ib)
            wss[r].copy_(ws)
    done += n
    torch.cuda.synchronize()
bad_out = (outs != ib_ref).any(2).any(1)
print(f"mode {MODE}: runs with wrong img_bias {int(bad_out.sum())} / {REPS}; ws ever wrong: "
      f"{int((wss != ws_ref).any(1).sum())}", flush=True)
gap_ref32 = (ws_ref.view(B, 16, Cc).sum(1) / (h * w))  # fp32 order differs: tolerance
for r in bad_out.nonzero().view(-1).tolist()[:8]:
    g = dbg[r, :, :Cc].double()
    pl = dbg[r, :, Cc:].double()
    gd = (g - part).abs()
    pd = (pl - pool_ref).abs()
    bi = (outs[r] != ib_ref).any(1).nonzero().view(-1).tolist()
    worst = gd.max(1)
    print(f"  run {r}: bad images {bi}; max |gap - ref| per image {[f'{v:.2e}' for v in worst.values.tolist()]} "
          f"at ch {worst.indices.tolist()}; max |pool - ref| {[f'{v:.2e}' for v in pd.max(1).values.tolist()]}",
          flush=True)
    for b in bi:
        bad_ch = (gd[b] > 1e-4).nonzero().view(-1).tolist()
        print(f"    image {b}: gap channels off {len(bad_ch)}: {bad_ch[:40]}", flush=True)
ok = (~bad_out).nonzero().view(-1).tolist()[:1]
for r in ok:
    print(f"  good run {r}: max |gap - ref| {(dbg[r, :, :Cc].double() - part).abs().max().item():.2e}")
