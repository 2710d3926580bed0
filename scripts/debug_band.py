"""Debug: where does fused_ir_band differ from its numpy emulation (per row / column)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_fused_band_cpu import band_block, pack_band
from semantic_segmentation_server_amd.ops import fused_band as FB

cin, cout, stride, H, W, R, nslot = [int(v) for v in sys.argv[1:8]]
blk, spec = band_block(cin, cout, stride, seed=1)
x = torch.randn(2, cin, H, W, generator=torch.Generator().manual_seed(3)).to(torch.bfloat16)
xn = x.permute(0, 2, 3, 1).contiguous()
packed = pack_band(blk, spec, device="cuda")
OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
out = torch.full((2, OH, OW, cout), float("nan"), dtype=torch.bfloat16, device="cuda")
FB.fused_ir_band(xn.cuda(), packed, out, B=2, IH=H, IW=W, stride=stride, residual=spec.residual, R=R, nslot=nslot)
torch.cuda.synchronize()
emu = FB.emulate_fused_band(xn.float().numpy(), packed, stride=stride, residual=spec.residual)
d = np.abs(out.float().cpu().numpy() - emu).max(axis=(0, 3))
bad = np.argwhere(d > 0.05)
print("max err", d.max(), "bad pixels", len(bad), "of", d.size)
print("bad rows", sorted(set(bad[:, 0].tolist()))[:40])
print("bad cols", sorted(set(bad[:, 1].tolist()))[:40])
