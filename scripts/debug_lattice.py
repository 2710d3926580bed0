"""Which output pixels a lattice-span launch leaves unwritten / non-finite: per span, the
output-list indices affected (GPU diagnostic for fused_ir_stream variant bit 8)."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from semantic_segmentation_server_amd.ops import fused_span as FS  # noqa: E402
from test_fused_span_cpu import _block, pack_block  # noqa: E402

DEV = "cuda"
for cout, S, B in ((160, 8, 1), (160, 8, 3), (320, 8, 1)):
    H = W = 33
    blk, spec = _block(160, cout, 2, seed=1)
    packed = pack_block(blk, spec, device=DEV)
    lt = FS.lattice_table(H, W, S, 2, DEV)
    x = torch.randn(B, H, W, 160).to(torch.bfloat16).to(DEV)
    for v in ((0, 1, 2, 4) if cout == 160 else (1,)):
        out = torch.full((B, H, W, cout), float("nan"), dtype=torch.bfloat16, device=DEV)
        FS.fused_ir_stream(x, packed, lt, out, B=B, residual=spec.residual, variant=v)
        torch.cuda.synchronize()
        bad = ~torch.isfinite(out.float()).all(-1).view(B, -1).cpu()
        tab = lt["table"].cpu().numpy()
        ol = lt["olist"]
        print(f"cout {cout} S {S} B {B} v {v}: {int(bad.sum())} bad of {B * H * W}")
        for b in range(B):
            for j in range(S):
                n = tab[j, 1]
                pix = tab[j, ol:ol + n] >> 12
                idx = [i for i in range(n) if bad[b, pix[i]]]
                if idx:
                    print(f"  b {b} span {j} n {n}: {len(idx)} bad, list idx {idx[:12]}{'...' if len(idx) > 12 else ''}")
