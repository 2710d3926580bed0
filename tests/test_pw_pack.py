"""CPU check of pw_conv's host-side weight packing: unpacking the packed tensor with
the kernel's own index formula (pw_conv.hip) must give back W and the bias."""
import pytest
import torch

from semantic_segmentation_server_amd.ops import hip_ops as K


@pytest.mark.parametrize("N,Kd,n_out", [(96, 160, None), (21, 256, 24), (576, 96, None), (144, 24, None)])
def test_pack_pw_roundtrip(N, Kd, n_out):
    g = torch.Generator().manual_seed(0)
    w = torch.randn(N, Kd, generator=g)
    b = torch.randn(N, generator=g)
    p = K.pack_pw_weights(w, b, N_out=n_out)
    Np = max(N, n_out or N)
    NC, KS = -(-Np // 64), -(-Kd // 32)
    assert p.dtype == torch.bfloat16 and p.numel() == NC * (4 * KS + 1) * 512
    chunks = p.reshape(NC, (4 * KS + 1) * 512)
    wrec = torch.zeros(NC * 64, KS * 32)
    brec = torch.zeros(NC * 64)
    for c in range(NC):
        wt = chunks[c, : 4 * KS * 512].float().reshape(4, KS, 64, 8)
        for j in range(4):
            for k in range(KS):
                for lane in range(64):
                    r, kq = lane % 16, lane // 16
                    wrec[c * 64 + j * 16 + r, k * 32 + kq * 8: k * 32 + kq * 8 + 8] = wt[j, k, lane]
        brec[c * 64:(c + 1) * 64] = chunks[c, 4 * KS * 512:].contiguous().view(torch.float32)[:64]
    assert torch.equal(wrec[:N, :Kd], w.to(torch.bfloat16).float())
    assert wrec[N:].abs().sum() == 0 and wrec[:, Kd:].abs().sum() == 0
    assert torch.equal(brec[:N], b) and brec[N:].abs().sum() == 0


def test_pw_supported():
    assert K.pw_supported(160, 960) and K.pw_supported(24, 144) and K.pw_supported(320, 256)
    assert not K.pw_supported(960, 160)  # deep K: the generic implicit GEMM handles it
    assert not K.pw_supported(256, 21)   # N must be padded to a multiple of 8


@pytest.mark.parametrize("B,H,W,dil,bm", [(2, 33, 33, 18, 128), (3, 33, 33, 6, 256), (1, 9, 7, 12, 128)])
def test_tap_group_perm_is_tap_uniform(B, H, W, dil, bm):
    """Every BM-row tile of the permutation holds pixels with one tap-validity pattern."""
    p = K.tap_group_perm(B, H, W, 3, dil, bm)
    assert p.numel() % bm == 0
    v = p[p >= 0]
    assert torch.equal(torch.sort(v).values, torch.arange(B * H * W, dtype=torch.int32))
    for t in range(p.numel() // bm):
        rows = p[t * bm:(t + 1) * bm]
        rows = rows[rows >= 0].long() % (H * W)
        if rows.numel() == 0:
            continue
        y, x = rows // W, rows % W
        pat = torch.stack([(y - dil >= 0), (y + dil < H), (x - dil >= 0), (x + dil < W)], 1)
        assert torch.all(pat == pat[0]), f"tile {t} mixes tap patterns"


def test_pack_tap_roundtrip():
    g = torch.Generator().manual_seed(1)
    Cout, Cin = 200, 160
    w = torch.randn(Cout, 3, 3, Cin, generator=g)
    b = torch.randn(Cout, generator=g)
    p, bp = K.pack_tap_weights(w, b)
    G, KS = 2, 5
    t5 = p.float().reshape(9, G, 8, KS, 64, 8)
    rec = torch.zeros(9, G * 128, KS * 32)
    for lane in range(64):
        r, kq = lane % 16, lane // 16
        for j in range(8):
            for k in range(KS):
                rec[:, j * 16 + r::128][:, :G, k * 32 + kq * 8:k * 32 + kq * 8 + 8] = t5[:, :, j, k, lane]
    want = w.to(torch.bfloat16).float().reshape(Cout, 9, Cin).permute(1, 0, 2)
    assert torch.equal(rec[:, :Cout, :Cin], want) and rec[:, Cout:].abs().sum() == 0
    assert torch.equal(bp[:Cout], b) and bp[Cout:].abs().sum() == 0


def test_pack_dw_proj_layout():
    g = torch.Generator().manual_seed(2)
    Cout, hid = 96, 192
    wp = torch.randn(Cout, hid, generator=g)
    wd9 = torch.randn(9, hid, generator=g)
    bd = torch.randn(hid, generator=g)
    p = K.pack_dw_proj(wp, wd9, bd)
    assert p.dtype == torch.float16
    NS, NC = Cout // 16, hid // 32
    chunks = p.reshape(NC, (NS + 1) * 512).float()
    for c in range(NC):
        frag = chunks[c, :NS * 512].reshape(NS, 64, 8)
        for n in range(NS):
            for lane in range(64):
                r, kq = lane % 16, lane // 16
                want = wp[n * 16 + r, c * 32 + kq * 8: c * 32 + kq * 8 + 8].half().float()
                assert torch.equal(frag[n, lane], want)
        dw = chunks[c, NS * 512:]
        assert torch.equal(dw[:288].reshape(9, 32), wd9[:, c * 32:(c + 1) * 32].half().float())
        assert torch.equal(dw[288:320], bd[c * 32:(c + 1) * 32].half().float())
        assert dw[320:].abs().sum() == 0
