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
NT = 256 if MODE & 4 else 512 if MODE & 8 else 1024
# reference: this mode's own kernel, run alone (summation order differs between modes)
H().aspp_pool(x.data_ptr(), ws.data_ptr(), w1t.data_ptr(), b1.data_ptr(), w2t.data_ptr(),
              ib.data_ptr(), B, h * w, Cc, N, torch.cuda.current_stream().cuda_stream, 0, MODE)
torch.cuda.synchronize()
ib_ref = ib.clone()
ws_ref = ws.clone()
part = ws_ref.view(B, -1, Cc).double().sum(1) / (h * w)
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
DS = Cc + N + 4 * 4 * NT
dbg = torch.zeros((REPS, B, DS), dtype=torch.float32, device="cuda")
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
gap_ref32 = (ws_ref.view(B, -1, Cc).sum(1) / (h * w))  # fp32 order differs: tolerance
w1d, w2d = w1t.double(), w2t.double()


def stage_expect(x, wt, K_):
    """per-thread float4 slice sums of stage with input vector x (K_ long), NT threads"""
    nq, nks = N // 4, NT // (N // 4)
    per = (K_ + nks - 1) // nks
    out = torch.zeros(NT, 4, dtype=torch.float64)
    for t in range(NT):
        ks, q = t // nq, t % nq
        k0 = min(K_, ks * per)
        k1 = min(K_, k0 + per)
        if k1 > k0:
            out[t] = (x[k0:k1, None] * wt[k0:k1, 4 * q:4 * q + 4]).sum(0)
    return out


for r in bad_out.nonzero().view(-1).tolist()[:6]:
    bi = (outs[r] != ib_ref).any(1).nonzero().view(-1).tolist()
    for b in bi:
        d = dbg[r, b].double().cpu()
        gap, pool = d[:Cc], d[Cc:Cc + N]
        v = d[Cc + N:Cc + N + 4 * NT * 4].view(4, NT, 4)
        e1 = stage_expect(gap, w1d.cpu(), Cc)
        e2 = stage_expect(pool, w2d.cpu(), N)
        reg1 = (v[0] - e1).abs().max(1).values
        lds1 = (v[1] - v[0]).abs().max(1).values
        reg2 = (v[2] - e2).abs().max(1).values
        lds2 = (v[3] - v[2]).abs().max(1).values
        def where(x, tol=1e-4):
            idx = (x > tol).nonzero().view(-1).tolist()
            return f"{len(idx)} threads (waves {sorted(set(i // 64 for i in idx))}) {idx[:8]}"
        print(f"  run {r} image {b}: stage1 reg-vs-expected {where(reg1)}; stage1 lds-view-vs-reg "
              f"{where(lds1)}; stage2 reg-vs-expected {where(reg2)}; stage2 lds-vs-reg {where(lds2)}",
              flush=True)
        bad_t = (reg1 > 1e-4).nonzero().view(-1).tolist()[:2] + (reg2 > 1e-4).nonzero().view(-1).tolist()[:2]
        for t in bad_t[:2]:
            print(f"     thread {t}: stage1 got {v[0][t].tolist()} want {e1[t].tolist()}", flush=True)
