"""Microbenchmark of one fused_ir_band configuration at B=32 (for rocprofv3 PMC passes):
python scripts/bench_band.py --block 1 --R 7 --nslot 1 --reps 5"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_fused_band_cpu import band_block, pack_band  # noqa: E402
from semantic_segmentation_server_amd.ops import fused_band as FB  # noqa: E402

BLOCKS = {1: (16, 24, 2, 257), 2: (24, 24, 1, 129), 3: (24, 32, 2, 129), 4: (32, 32, 1, 65),
          6: (32, 64, 2, 65)}
p = argparse.ArgumentParser()
p.add_argument("--block", type=int, default=1)
p.add_argument("--R", type=int, default=7)
p.add_argument("--nslot", type=int, default=1)
p.add_argument("--B", type=int, default=32)
p.add_argument("--reps", type=int, default=5)
a = p.parse_args()
cin, cout, stride, H = BLOCKS[a.block]
blk, spec = band_block(cin, cout, stride, seed=1)
packed = pack_band(blk, spec, device="cuda")
x = torch.randn(a.B, H, H, cin, device="cuda").to(torch.bfloat16)
OH = (H - 1) // stride + 1
out = torch.empty(a.B, OH, OH, cout, device="cuda", dtype=torch.bfloat16)
for _ in range(2):
    FB.fused_ir_band(x, packed, out, B=a.B, IH=H, IW=H, stride=stride, residual=spec.residual, R=a.R,
                     nslot=a.nslot)
torch.cuda.synchronize()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(a.reps):
    FB.fused_ir_band(x, packed, out, B=a.B, IH=H, IW=H, stride=stride, residual=spec.residual, R=a.R,
                     nslot=a.nslot)
en.record()
en.synchronize()
print(f"block{a.block} R={a.R} nslot={a.nslot}: {st.elapsed_time(en) / a.reps * 1e3:.1f} us")
