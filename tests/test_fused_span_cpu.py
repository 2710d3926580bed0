"""CPU tier for the fused inverted-residual span kernel's host side (ops/fused_span.py):
the span/halo table and the chunk-image packing are checked by re-executing the
kernel's data flow in numpy from the packed bytes, against the torch block (fp32)."""
import numpy as np
import pytest
import torch

from semantic_segmentation_server_amd.models.layers import init_random
from semantic_segmentation_server_amd.models.mobilenetv2 import InvertedResidual, IRSpec
from semantic_segmentation_server_amd.ops import fused_span as FS


@pytest.mark.parametrize("H,W,S,dil", [(33, 33, 8, 1), (33, 33, 8, 2), (17, 19, 3, 2), (33, 33, 16, 1)])
def test_span_table_covers_every_tap(H, W, S, dil):
    t = FS.span_table(H, W, S, dil)
    tab = t["table"].numpy()
    WCP, WR = t["WCP"], t["WR"]
    covered = np.zeros(H * W, dtype=int)
    for j in range(S):
        p0, p1, wy0, nh = tab[j, :4]
        covered[p0:p1] += 1
        assert p1 - p0 <= 144
        ent = tab[j, 4:4 + nh]
        px, pos = ent >> 12, ent & 4095
        assert len(set(pos.tolist())) == nh                     # one slot per halo pixel
        assert pos.max() < WR * WCP - 1                          # the dummy slot stays free
        halo = dict(zip(pos.tolist(), px.tolist()))
        for p in range(p0, p1):
            y, x = divmod(p, W)
            for dy in (-dil, 0, dil):
                for dx in (-dil, 0, dil):
                    yy, xx = y + dy, x + dx
                    wpos = (yy - wy0) * WCP + xx + dil
                    assert 0 <= wpos < WR * WCP
                    if 0 <= yy < H and 0 <= xx < W:
                        assert halo.get(wpos) == yy * W + xx      # in-image tap: computed
                    else:
                        assert wpos not in halo                   # padding tap: stays zero
    assert (covered == 1).all()
    assert -(-t["nh_max"] // 16) <= 8 * t["xg"]


def _block(cin, cout, dil, seed):
    spec = IRSpec(cin, cout, 6, 1, dil)
    blk = InvertedResidual(spec)
    init_random(blk, seed=seed)
    for m in blk.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 2.0)
    return blk.eval(), spec


def pack_block(blk, spec, device=None):
    ew, eb = blk.expand.fold()
    dwf, dbf = blk.dw.fold()
    pwf, pbf = blk.project.fold()
    return FS.pack_fused_span(ew[:, :, 0, 0], eb, dwf[:, 0], dbf, pwf[:, :, 0, 0], pbf, Cin=spec.cin,
                              hid=spec.hidden, Cout=spec.cout, device=device)


@pytest.mark.parametrize("cin,cout,dil,H,S", [(64, 64, 1, 13, 2), (64, 96, 1, 11, 1), (96, 160, 1, 9, 1),
                                              (160, 160, 2, 12, 2), (160, 320, 2, 9, 1)])
def test_packed_span_emulation_matches_block(cin, cout, dil, H, S):
    blk, spec = _block(cin, cout, dil, seed=cin + cout + dil)
    g = torch.Generator().manual_seed(5)
    B, W = 1, H + 2
    x = torch.randn(B, cin, H, W, generator=g).to(torch.bfloat16).float()
    with torch.no_grad():
        ref = blk(x).permute(0, 2, 3, 1).numpy()
    packed = pack_block(blk, spec)
    table = FS.span_table(H, W, S, dil)
    got = FS.emulate_fused_span(x.permute(0, 2, 3, 1).numpy(), packed, table, residual=spec.residual)
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert rel < 1e-2, rel


@pytest.mark.parametrize("H,W,S", [(33, 33, 8), (33, 33, 16), (12, 33, 3), (17, 19, 3), (4, 33, 1)])
def test_lattice_table_covers_every_tap(H, W, S):
    """Lattice spans (dilation 2): every output pixel exactly once; each of its 9 taps, in
    window coordinates (dilation 1, pitch WCP), is the halo slot of the right pixel when
    the dilated tap is in the image and an unwritten (zero) slot when it is not."""
    dil = 2
    t = FS.lattice_table(H, W, S, dil)
    tab = t["table"].numpy()
    WCP, WR, ol = t["WCP"], t["WR"], t["olist"]
    covered = np.zeros(H * W, dtype=int)
    for j in range(S):
        p0, n, _wy0, nh = tab[j, :4]
        assert p0 == 0 and 0 < n <= 144
        ent = tab[j, 4:4 + nh]
        px, pos = ent >> 12, ent & 4095
        assert len(set(pos.tolist())) == nh
        assert pos.max() < WR * WCP - 1
        halo = dict(zip(pos.tolist(), px.tolist()))
        oe = tab[j, ol:ol + n]
        for p, c in zip((oe >> 12).tolist(), (oe & 4095).tolist()):
            covered[p] += 1
            y, x = divmod(p, W)
            for t9 in range(9):
                dy, dx = t9 // 3 - 1, t9 % 3 - 1
                w = c + dy * WCP + dx
                assert 0 <= w < WR * WCP - 1
                yy, xx = y + dil * dy, x + dil * dx
                if 0 <= yy < H and 0 <= xx < W:
                    assert halo.get(w) == yy * W + xx
                else:
                    assert w not in halo
    assert (covered == 1).all()
    assert t["nh_max"] <= FS.LAT_XQ * 64 or (H, W) != (33, 33)


@pytest.mark.parametrize("cin,cout,H,S", [(160, 160, 12, 3), (160, 320, 4, 1), (160, 160, 33, 8)])
def test_lattice_emulation_matches_block(cin, cout, H, S):
    blk, spec = _block(cin, cout, 2, seed=cin + cout + 7)
    g = torch.Generator().manual_seed(6)
    B, W = 1, 33
    x = torch.randn(B, cin, H, W, generator=g).to(torch.bfloat16).float()
    with torch.no_grad():
        ref = blk(x).permute(0, 2, 3, 1).numpy()
    packed = pack_block(blk, spec)
    xh = x.permute(0, 2, 3, 1).numpy()
    got = FS.emulate_fused_span(xh, packed, FS.lattice_table(H, W, S, 2), residual=spec.residual)
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert rel < 1e-2, rel
    # the same fp16 chain per pixel as the raster spans: identical results
    ras = FS.emulate_fused_span(xh, packed, FS.span_table(H, W, S, 2), residual=spec.residual)
    assert np.array_equal(got, ras)
