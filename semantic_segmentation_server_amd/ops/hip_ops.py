"""Checked torch-tensor wrappers around the gfx950 kernels in ``_hip``.

Every wrapper validates dtype/contiguity/shape on the host (an out-of-bounds
kernel can reset the whole GPU node, so shapes are checked before launch), then
launches on ``torch.cuda.current_stream()`` — inside a ``torch.cuda.graph``
capture that is the capture stream, so the launches are recorded into the graph.
"""
from __future__ import annotations

from typing import List, Optional

import os

import torch

from .native import hip as _hip_mod

ACT = {None: 0, "none": 0, "relu": 1, "relu6": 2}


_DEBUG_SYNC = os.environ.get("SSA_DEBUG_SYNC", "0") == "1"


def _stream() -> int:
    # the raw handle of the current stream by two C calls (utils/fast_cuda.py: the
    # torch.cuda.current_stream() path resolves the device on every launch)
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def _dbg(name: str, **shapes) -> None:
    """SSA_DEBUG_SYNC=1: synchronise after every launch and name the failing kernel."""
    if not _DEBUG_SYNC or torch.cuda.is_current_stream_capturing():
        return
    try:
        torch.cuda.synchronize()
    except Exception as e:
        raise RuntimeError(f"kernel {name} failed with {shapes}: {e}") from e


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _chk(t: torch.Tensor, dtype, name: str, numel: Optional[int] = None) -> None:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a CUDA tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if numel is not None and t.numel() < numel:
        raise ValueError(f"{name}: has {t.numel()} elements, kernel needs {numel}")


def conv_out_hw(IH: int, IW: int, k: int, stride: int, dil: int):
    pad = dil * (k // 2)
    OH = (IH + 2 * pad - dil * (k - 1) - 1) // stride + 1
    OW = (IW + 2 * pad - dil * (k - 1) - 1) // stride + 1
    return OH, OW


def conv_gemm(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, out: torch.Tensor, *,
              B: int, IH: int, IW: int, Cin: int, OH: int, OW: int, Cout: int, k: int = 1,
              stride: int = 1, dil: int = 1, ldo: Optional[int] = None, co_off: int = 0,
              act=None, res: Optional[torch.Tensor] = None, ldr: Optional[int] = None,
              img_bias: Optional[torch.Tensor] = None, variant: int = 0,
              perm: Optional[torch.Tensor] = None) -> torch.Tensor:
    """NHWC implicit-GEMM conv (variant: 0 auto, 1 register-fed, 2 LDS-staged, 3/4 LDS-DMA
    3/2-stage, 5/6 LDS-DMA 128x256/256x256). x: [B,IH,IW,Cin] bf16; w: [Cout,k,k,Cin] bf16;
    out: [B,OH,OW,ldo] bf16 written at channel offset co_off. ``perm`` (int32, from
    ``tap_group_perm``) reorders the GEMM rows so that tiles hold pixels of equal tap
    validity (LDS-DMA variants only)."""
    ldo = Cout if ldo is None else ldo
    ldr = Cout if ldr is None else ldr
    if Cin % 8:
        raise ValueError("conv_gemm: Cin must be a multiple of 8")
    if co_off + Cout > ldo:
        raise ValueError("conv_gemm: co_off + Cout > ldo")
    _chk(x, torch.bfloat16, "x", B * IH * IW * Cin)
    _chk(w, torch.bfloat16, "w", Cout * k * k * Cin)
    _chk(bias, torch.float32, "bias", Cout)
    _chk(out, torch.bfloat16, "out", B * OH * OW * ldo)
    if res is not None:
        _chk(res, torch.bfloat16, "res", B * OH * OW * ldr)
    if img_bias is not None:
        _chk(img_bias, torch.float32, "img_bias", B * Cout)
    Mp = 0
    if perm is not None:
        _chk(perm, torch.int32, "perm")
        Mp = perm.numel()
        if variant not in (3, 4, 5, 6, 8, 9, 10):
            raise ValueError("conv_gemm: perm needs an LDS-DMA variant (3-6, 8-10)")
        # every entry must be a valid pixel or -1 (checked once per tensor, host side)
        if not getattr(perm, "_ssa_checked", False):
            pc = perm.cpu()
            if pc.min().item() < -1 or pc.max().item() >= B * OH * OW:
                raise ValueError("conv_gemm: perm entry out of range")
            perm._ssa_checked = True
    _hip_mod().conv_gemm(_ptr(x), _ptr(w), _ptr(bias), _ptr(img_bias), _ptr(res), _ptr(out), B, IH,
                         IW, Cin, OH, OW, Cout, k, k, stride, dil, ldo, co_off, ldr, ACT[act],
                         _stream(), variant, _ptr(perm), Mp)
    _dbg('conv_gemm')
    return out


def tap_group_perm(B: int, H: int, W: int, k: int, dil: int, BM: int, device=None) -> torch.Tensor:
    """GEMM-row permutation for a stride-1 dilated kxk conv on B x H x W maps.

    Pixels are grouped by which of their taps fall inside the image (per axis: is
    the -dil*(k//2) and the +dil*(k//2) neighbour inside), each group padded with -1
    rows to a multiple of the tile height BM. Every tile is then tap-uniform, so
    the kernel's per-tile tap mask skips all padding taps: for the ASPP rates
    6/12/18 on 33x33 maps 6.95/5.17/3.64 of 9 taps are live on average, against
    ~8/7/6 with tiles cut from raster order. Within a group the raster order
    (image, row, column) is kept for locality."""
    r = dil * (k // 2)

    def cls(n):
        i = torch.arange(n)
        return (i - r < 0).long() * 2 + (i + r > n - 1).long()

    key = (cls(H)[:, None] * 4 + cls(W)[None, :]).reshape(-1)  # [H*W]
    order = []
    for c in torch.unique(key).tolist():
        px = torch.nonzero(key == c).flatten()
        idx = (torch.arange(B)[:, None] * (H * W) + px[None, :]).reshape(-1)
        pad = (-idx.numel()) % BM
        order.append(idx)
        if pad:
            order.append(torch.full((pad,), -1, dtype=torch.long))
    return torch.cat(order).to(torch.int32).to(device).contiguous()


GROUP_TILE = {5: (128, 256), 6: (256, 256), 8: (128, 256), 10: (128, 128), 11: (128, 128),
              12: (256, 256), 13: (128, 256), 14: (256, 256), 15: (256, 256), 16: (256, 256),
              17: (128, 256), 18: (256, 128)}


def _tile_taps(B: int, H: int, W: int, k: int, dil: int, BM: int,
               perm: Optional[torch.Tensor]) -> torch.Tensor:
    """Live taps per BM-row tile of a stride-1 'same' kxk conv's GEMM (the union of
    the in-image taps of the tile's rows, as the kernel's per-tile tap mask)."""
    r = dil * (k // 2)
    ys, xs = torch.arange(H), torch.arange(W)
    bits = torch.zeros(H, W, dtype=torch.long)
    for t in range(k * k):
        dy, dx = (t // k) * dil - r, (t % k) * dil - r
        oky = ((ys + dy >= 0) & (ys + dy < H))[:, None]
        okx = ((xs + dx >= 0) & (xs + dx < W))[None, :]
        bits |= (oky & okx).long() << t
    rows = bits.reshape(-1).repeat(B)  # [B*H*W], raster GEMM rows
    if perm is not None:
        pc = perm.cpu().long()
        rows = torch.where(pc >= 0, rows[pc.clamp(min=0)], torch.zeros_like(pc))
    pad = (-rows.numel()) % BM
    rows = torch.cat([rows, torch.zeros(pad, dtype=torch.long)]).reshape(-1, BM)
    tile = torch.zeros(rows.shape[0], dtype=torch.long)
    for j in range(BM):  # bitwise OR-reduce over the tile's rows
        tile |= rows[:, j]
    return sum(((tile >> t) & 1) for t in range(k * k))


def grouped_tile_order(convs: List[dict], variant: int, device=None, xcds: int = 1, ks: int = 1) -> torch.Tensor:
    """Block -> tile table of ``conv_gemm_grouped``: every tile of every conv as
    (group << 24) | tile, heaviest first (work = live taps x 64-channel K chunks;
    longest-processing-time order, so the short 1x1 / edge tiles fill the tail).

    ``xcds > 1`` (8 on MI355X): block i runs on XCD i % xcds, so each XCD gets one
    contiguous run of every conv's row tiles (LPT order inside it) -- a dilated
    tile's shifted-tap rows belong to its neighbour tiles, which then sit in the
    same XCD's L2 instead of being fetched from MALL by all eight."""
    BM, BN = GROUP_TILE[variant]
    ent, cost, part = [], [], []
    for g, c in enumerate(convs):
        tn = -(-c["Cout"] // BN)
        taps = _tile_taps(c["B"], c["OH"], c["OW"], c["k"], c["dil"], BM, c.get("perm"))
        kch = -(-c["Cin"] // 64)
        ntm = taps.numel()
        for tm in range(ntm):
            for n in range(tn):
                stages = int(taps[tm]) * kch
                for sl in range(ks):  # K slice sl runs stages [sl*S/ks, (sl+1)*S/ks) (split-K)
                    ent.append((g << 24) | (sl << 20) | (tm * tn + n))
                    cost.append((sl + 1) * stages // ks - sl * stages // ks)
                    part.append(min(xcds - 1, tm * xcds // max(1, ntm)))
    if xcds <= 1:
        idx = sorted(range(len(ent)), key=lambda i: (-cost[i], i))
        return torch.tensor([ent[i] for i in idx], dtype=torch.int32).to(device).contiguous()
    lists = [sorted((i for i in range(len(ent)) if part[i] == x), key=lambda i: (-cost[i], i))
             for x in range(xcds)]
    out, j = [], 0
    while any(j < len(lst) for lst in lists):
        for x in range(xcds):  # position 8j + x runs on XCD x
            if j < len(lists[x]):
                out.append(ent[lists[x][j]])
            else:  # this XCD's run is exhausted: lend the slot to the longest remaining run
                donor = max(range(xcds), key=lambda y: len(lists[y]) - j)
                if len(lists[donor]) > j + 1:
                    out.append(ent[lists[donor].pop()])
        j += 1
    assert sorted(out) == sorted(ent)
    return torch.tensor(out, dtype=torch.int32).to(device).contiguous()


def grouped_tile_order_branch(convs: List[dict], variant: int, device=None, xcds: int = 8) -> torch.Tensor:
    """Branch-affine block -> tile table: every XCD (block i runs on XCD i % xcds under the
    round-robin dispatch; speed only, never correctness) is given tiles of ONE conv, so that
    conv's weights (1.47 MB per 3x3 ASPP branch: re-read by every row tile) stay in the XCD's
    4 MiB L2 instead of four branches' 4.4 MB thrashing every L2 (the global LPT order mixes
    branches on every XCD; the row-range split of ``grouped_tile_order(xcds=8)`` did too).
    Each XCD runs the same number of blocks (positional dispatch); 3x3 convs get XCD sets
    in proportion to their work, 1x1 tiles fill the remaining block counts of the least
    loaded XCDs; each XCD runs its tiles heaviest first."""
    BM, BN = GROUP_TILE[variant]
    tiles = []  # (cost, entry, group)
    for g, c in enumerate(convs):
        tn = -(-c["Cout"] // BN)
        taps = _tile_taps(c["B"], c["OH"], c["OW"], c["k"], c["dil"], BM, c.get("perm"))
        kch = -(-c["Cin"] // 64)
        for tm in range(taps.numel()):
            for n in range(tn):
                tiles.append((int(taps[tm]) * kch, (g << 24) | (tm * tn + n), g))
    G = len(convs)
    return _branch_affine(tiles, [g for g in range(G) if convs[g]["k"] > 1] or list(range(G)), xcds, device)


def _branch_affine(tiles, heavy, xcds, device):
    """XCD assignment of ``grouped_tile_order_branch``. tiles: (cost, entry, key); each key in
    ``heavy`` (a weight slab: a 3x3 conv, or one of its channel tiles) gets an XCD set."""
    # the dispatcher hands block i to XCD i % xcds whatever its load, so every XCD runs the
    # same NUMBER of blocks: the 3x3 branches get XCD sets in proportion to their work, and
    # the light 1x1 tiles (164 KB of weights) fill every XCD's remaining block count
    gcost = {g: sum(t[0] for t in tiles if t[2] == g) for g in heavy}
    tot = max(1, sum(gcost.values()))
    share = {g: xcds * gcost[g] / tot for g in heavy}
    cnt = {g: max(1, int(share[g])) for g in heavy}
    while sum(cnt.values()) > xcds:
        i = max((g for g in heavy if cnt[g] > 1), key=lambda g: cnt[g] - share[g])
        cnt[i] -= 1
    while sum(cnt.values()) < xcds:
        i = max(heavy, key=lambda g: share[g] - cnt[g])
        cnt[i] += 1
    xs, x0 = {}, 0
    for g in heavy:
        xs[g] = list(range(x0, x0 + cnt[g]))
        x0 += cnt[g]
    T = len(tiles)
    cap = [T // xcds + (1 if x < T % xcds else 0) for x in range(xcds)]
    lists = [[] for _ in range(xcds)]
    load = [0] * xcds
    order = sorted(tiles, key=lambda t: (-t[0], t[1]))
    for cost, ent, g in order:
        if g not in xs:
            continue
        cands = [y for y in xs[g] if len(lists[y]) < cap[y]] or [y for y in range(xcds) if len(lists[y]) < cap[y]]
        x = min(cands, key=lambda y: load[y])
        lists[x].append((cost, ent))
        load[x] += cost
    for cost, ent, g in order:  # fillers: the least loaded XCD with blocks left
        if g in xs:
            continue
        x = min((y for y in range(xcds) if len(lists[y]) < cap[y]), key=lambda y: load[y])
        lists[x].append((cost, ent))
        load[x] += cost
    for lst in lists:
        lst.sort(key=lambda t: (-t[0], t[1]))
    out = []
    for j in range(max(cap)):
        for x in range(xcds):  # position xcds * j + x runs on XCD x
            if j < len(lists[x]):
                out.append(lists[x][j][1])
    assert sorted(out) == sorted(t[1] for t in tiles)
    return torch.tensor(out, dtype=torch.int32).to(device).contiguous()


def conv_gemm_grouped(convs: List[dict], order: torch.Tensor, variant: int = 5, ks: int = 1,
                      part: Optional[torch.Tensor] = None, bias_cat: Optional[torch.Tensor] = None,
                      cnt: Optional[torch.Tensor] = None) -> None:
    """Up to 4 independent stride-1 'same' NHWC convs with one Cout (the ASPP branches)
    in ONE LDS-DMA grid, tiles in the ``grouped_tile_order`` table. Each conv is a
    dict of conv_gemm's arguments: x, w, bias, out, B, IH, IW, Cin, OH, OW, Cout, k,
    dil, ldo, co_off, act, and optionally perm (tap_group_perm with the variant's BM).

    ``ks`` > 1 (split-K, small batches): the order table (``grouped_tile_order(..., ks=)``)
    carries ks K slices per tile; their fp32 partials go to ``part`` [ks, B*OH*OW, ldo]
    and stream_combine adds them, ``bias_cat`` (the branches' biases at their co_off) and
    the shared activation into ``out``: the convs must tile [0, ldo) of one output. With
    ``cnt`` (int32, >= 4 x the largest conv's tile count, zeroed once: the last arriver of
    each tile resets its word) the tile's last arriving K slice does that sum inside the
    launch (no combine kernel; ``bias_cat`` is then unused)."""
    if not 1 <= len(convs) <= 4:
        raise ValueError("conv_gemm_grouped: 1..4 convs")
    if variant not in GROUP_TILE:
        raise ValueError(f"conv_gemm_grouped: variant must be one of {sorted(GROUP_TILE)}")
    BM, BN = GROUP_TILE[variant]
    tiles = []
    groups = []
    for c in convs:
        B, IH, IW, Cin, OH, OW, Cout, k = (c[n] for n in ("B", "IH", "IW", "Cin", "OH", "OW", "Cout", "k"))
        dil, ldo, co_off = c.get("dil", 1), c.get("ldo", Cout), c.get("co_off", 0)
        if Cin % 8 or k * k > 16 or Cout != convs[0]["Cout"] or (OH, OW) != (IH, IW):
            raise ValueError("conv_gemm_grouped: stride-1 'same' convs, Cin % 8 == 0, <= 16 taps, one Cout")
        if co_off + Cout > ldo:
            raise ValueError("conv_gemm_grouped: co_off + Cout > ldo")
        _chk(c["x"], torch.bfloat16, "x", B * IH * IW * Cin)
        _chk(c["w"], torch.bfloat16, "w", Cout * k * k * Cin)
        _chk(c["bias"], torch.float32, "bias", Cout)
        _chk(c["out"], torch.bfloat16, "out", B * OH * OW * ldo)
        perm = c.get("perm")
        Mp = 0
        if perm is not None:
            _chk(perm, torch.int32, "perm")
            Mp = perm.numel()
            if Mp % BM:
                raise ValueError("conv_gemm_grouped: perm rows must be a multiple of the tile height")
            if not getattr(perm, "_ssa_checked", False):
                pc = perm.cpu()
                if pc.min().item() < -1 or pc.max().item() >= B * OH * OW:
                    raise ValueError("conv_gemm_grouped: perm entry out of range")
                perm._ssa_checked = True
        M = Mp or B * OH * OW
        tiles.append(-(-M // BM) * -(-Cout // BN))
        groups.append((_ptr(c["x"]), _ptr(c["w"]), _ptr(c["bias"]), 0, 0, _ptr(c["out"]), B, IH, IW,
                       Cin, OH, OW, Cout, k, k, 1, dil, ldo, co_off, Cout, ACT[c.get("act")],
                       _ptr(perm), Mp))
    _chk(order, torch.int32, "order")
    if not getattr(order, "_ssa_checked", False):  # every block maps to a real tile
        oc = order.cpu().long()
        g, t, sl = oc >> 24, oc & 0xFFFFF, (oc >> 20) & 15
        lim = torch.tensor(tiles)[g.clamp(0, len(tiles) - 1)]
        if (g < 0).any() or (g >= len(convs)).any() or (t >= lim).any() or (sl >= ks).any():
            raise ValueError("conv_gemm_grouped: order entry out of range")
        if oc.numel() != sum(tiles) * ks:
            raise ValueError("conv_gemm_grouped: the order table must list every tile's K slices once")
        order._ssa_checked = True
    if ks > 1:
        c0 = convs[0]
        ldo, Mo = c0.get("ldo", c0["Cout"]), c0["B"] * c0["OH"] * c0["OW"]
        if part is None or bias_cat is None:
            raise ValueError("conv_gemm_grouped: split-K needs part and bias_cat")
        if len({c.get("act") for c in convs}) != 1 or c0.get("act") not in (None, "relu"):
            raise ValueError("conv_gemm_grouped: split-K needs one activation (none / relu)")
        if sorted(c.get("co_off", 0) for c in convs) != list(range(0, ldo, c0["Cout"])):
            raise ValueError("conv_gemm_grouped: split-K convs must tile the output channels")
        if any(c["out"].data_ptr() != c0["out"].data_ptr() or c.get("ldo", c["Cout"]) != ldo for c in convs):
            raise ValueError("conv_gemm_grouped: split-K convs must share one output")
        _chk(part, torch.float32, "part", ks * Mo * ldo)
        _chk(bias_cat, torch.float32, "bias_cat", ldo)
        if cnt is not None:
            _chk(cnt, torch.int32, "cnt", 4 * max(tiles))
    _hip_mod().conv_gemm_grouped(groups, _ptr(order), order.numel(), variant, _stream(), int(ks),
                                 _ptr(part) if ks > 1 else 0, _ptr(cnt) if (ks > 1 and cnt is not None) else 0,
                                 max(tiles))
    _dbg('conv_gemm_grouped')
    if ks > 1 and cnt is None:
        _hip_mod().stream_combine(_ptr(part), _ptr(bias_cat), 0, _ptr(c0["out"]), int(ks), Mo, ldo, _stream(),
                                  1 if c0.get("act") == "relu" else 0)
        _dbg('stream_combine')


def bias_act(x, bias, out, *, M: int, N: int, HW: int = 1, img_bias=None, act=None):
    """out[m, n] = act(x[m, n] + bias[n] + img_bias[m // HW][n]); x, out [M, N] bf16."""
    _chk(x, torch.bfloat16, "x", M * N)
    _chk(out, torch.bfloat16, "out", M * N)
    _chk(bias, torch.float32, "bias", N)
    if img_bias is not None:
        _chk(img_bias, torch.float32, "img_bias", (M // HW) * N)
        if M % HW:
            raise ValueError("bias_act: M must be a multiple of HW")
    if N % 8:
        raise ValueError("bias_act: N must be a multiple of 8")
    _hip_mod().bias_act(_ptr(x), _ptr(bias), _ptr(img_bias), _ptr(out), M, N, HW, ACT[act], _stream())
    _dbg('bias_act')
    return out


def pw_supported(K: int, N: int) -> bool:
    """True if pw_conv has an instantiation for this (K = Cin, N = Cout) pair."""
    ks = (K + 31) // 32
    return K % 8 == 0 and N % 8 == 0 and (ks <= 5 or ks in (8, 10))


def pack_pw_weights(w: torch.Tensor, bias: torch.Tensor, N_out: Optional[int] = None) -> torch.Tensor:
    """[N, K] (or [N, 1, 1, K]) weights + [N] fp32 bias -> pw_conv's packed operand.

    Per 64-output-channel chunk c: the weights in MFMA fragment order
    [4 subtiles][ceil(K/32)][64 lanes][8] bf16, element (j, k, lane, e) =
    W[c*64 + j*16 + lane%16][k*32 + (lane//16)*8 + e], then 1 KiB holding the
    chunk's 64 fp32 biases (zero-padded). ``N_out`` pads the channel count (e.g. 21
    logits written as 24)."""
    w = w.reshape(w.shape[0], -1).float()
    N, Kd = w.shape
    Np = max(N, N_out or N)
    NC, KS = -(-Np // 64), -(-Kd // 32)
    full = torch.zeros(NC * 64, KS * 32, dtype=torch.float32, device=w.device)
    full[:N, :Kd] = w
    # [c, j, r, k, kq, e] -> [c, j, k, kq, r, e]  (lane = kq*16 + r)
    wt = full.reshape(NC, 4, 16, KS, 4, 8).permute(0, 1, 3, 4, 2, 5).reshape(NC, -1)
    bt = torch.zeros(NC, 256, dtype=torch.float32, device=w.device)
    bflat = torch.zeros(NC * 64, dtype=torch.float32, device=w.device)
    bflat[:N] = bias.float().to(w.device)
    bt[:, :64] = bflat.reshape(NC, 64)
    return torch.cat([wt.to(torch.bfloat16), bt.view(torch.bfloat16)], dim=1).contiguous()


def pw_conv(x, wpk, out, *, M, K, N, ldo=None, co_off=0, act=None, res=None, ldr=None,
            img_bias=None, HW=1, mt=2, nch=1) -> torch.Tensor:
    """Weight-streamed 1x1 conv (pw_conv.hip). x: [M, K] bf16 (NHWC pixels), wpk from
    ``pack_pw_weights`` (weights + bias), out [M, ldo] bf16 (or fp16: written as fp16)
    at channel offset co_off."""
    ldo = N if ldo is None else ldo
    ldr = N if ldr is None else ldr
    if not pw_supported(K, N) or ldo % 8 or co_off % 8 or (res is not None and ldr % 8):
        raise ValueError(f"pw_conv: unsupported K={K} N={N} ldo={ldo} co_off={co_off}")
    if co_off + N > ldo or mt not in (2, 4) or nch < 1:
        raise ValueError("pw_conv: bad co_off / mt / nch")
    NC, KS = -(-N // 64), -(-K // 32)
    _chk(x, torch.bfloat16, "x", M * K)
    _chk(wpk, torch.bfloat16, "wpk", NC * (4 * KS + 1) * 512)
    out_f16 = out.dtype == torch.float16
    _chk(out, torch.float16 if out_f16 else torch.bfloat16, "out", M * ldo)
    if res is not None:
        _chk(res, torch.bfloat16, "res", M * ldr)
    if img_bias is not None:
        _chk(img_bias, torch.float32, "img_bias", (M // HW) * N)
        if M % HW:
            raise ValueError("pw_conv: M must be a multiple of HW with img_bias")
    _hip_mod().pw_conv(_ptr(x), _ptr(wpk), _ptr(img_bias), _ptr(res), _ptr(out), M, K, N, HW, ldo,
                       co_off, ldr, ACT[act], mt, nch, _stream(), int(out_f16))
    _dbg('pw_conv')
    return out


TAP_GROUP = 128  # output channels per tap_conv workgroup (tap_conv_group_channels())
TAP_CIN = (64, 128, 160, 256, 320)


def pack_tap_weights(w: torch.Tensor, bias: torch.Tensor):
    """[Cout, kh, kw, Cin] weights + [Cout] bias -> (packed bf16, padded fp32 bias) for
    tap_conv: [tap][ceil(Cout/128)][8 subtiles][ceil(Cin/32)][64 lanes][8], element
    (t, g, j, k, lane, e) = W[g*128 + j*16 + lane%16][t][k*32 + (lane//16)*8 + e]."""
    Cout, kh, kw, Cin = w.shape
    T, G, KS = kh * kw, -(-Cout // TAP_GROUP), -(-Cin // 32)
    full = torch.zeros(T, G * TAP_GROUP, KS * 32, dtype=torch.float32, device=w.device)
    full[:, :Cout, :Cin] = w.float().reshape(Cout, T, Cin).permute(1, 0, 2)
    # [t, g, j, r, k, kq, e] -> [t, g, j, k, kq, r, e]
    packed = full.reshape(T, G, 8, 16, KS, 4, 8).permute(0, 1, 2, 4, 5, 3, 6).contiguous()
    b = torch.zeros(G * TAP_GROUP, dtype=torch.float32, device=w.device)
    b[:Cout] = bias.float()
    return packed.to(torch.bfloat16).reshape(-1), b


def tap_conv(x, wpk, bias_p, out, *, B, H, W, Cin, Cout, k=3, dil=1, ldo=None, co_off=0, act=None,
             perm: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Dilated kxk stride-1 conv (tap_conv.hip). x [B,H,W,Cin] bf16; (wpk, bias_p) from
    ``pack_tap_weights``; out [B,H,W,ldo] at channel offset co_off; ``perm`` from
    ``tap_group_perm(B, H, W, k, dil, 256)`` groups tap-uniform 256-pixel tiles."""
    ldo = Cout if ldo is None else ldo
    if Cin not in TAP_CIN or Cout % 8 or ldo % 8 or co_off % 8 or co_off + Cout > ldo:
        raise ValueError(f"tap_conv: unsupported Cin={Cin} Cout={Cout} ldo={ldo} co_off={co_off}")
    G = -(-Cout // TAP_GROUP)
    _chk(x, torch.bfloat16, "x", B * H * W * Cin)
    _chk(wpk, torch.bfloat16, "wpk", k * k * G * TAP_GROUP * (-(-Cin // 32)) * 32)
    _chk(bias_p, torch.float32, "bias", G * TAP_GROUP)
    _chk(out, torch.bfloat16, "out", B * H * W * ldo)
    Mp = 0
    if perm is not None:
        _chk(perm, torch.int32, "perm")
        Mp = perm.numel()
        if not getattr(perm, "_ssa_checked", False):
            pc = perm.cpu()
            if pc.min().item() < -1 or pc.max().item() >= B * H * W:
                raise ValueError("tap_conv: perm entry out of range")
            perm._ssa_checked = True
    _hip_mod().tap_conv(_ptr(x), _ptr(wpk), _ptr(bias_p), _ptr(out), _ptr(perm), Mp, B, H, W, Cin,
                        Cout, k, k, dil, ldo, co_off, ACT[act], _stream())
    _dbg('tap_conv')
    return out


def fused_ir(x, packed: dict, out, *, B, IH, IW, OH, OW, tile=None, trace=None):
    """Fused inverted residual. ``packed`` from ``pack_fused_ir``.

    ``tile=(TY, TX)`` selects the general 2-D tile kernel (any dilation, Cin <= 160,
    Cout <= 320); ``None`` the 16-wide row-tile kernel (dilation 1, Cin <= 64)."""
    P = packed
    TY, TX = tile if tile is not None else (0, 0)
    if tile is None and P.get("dil", 1) != 1:
        raise ValueError("fused_ir: dilated blocks need the tile kernel")
    _chk(x, torch.bfloat16, "x", B * IH * IW * P["Cin"])
    _chk(out, torch.bfloat16, "out", B * OH * OW * P["Cout"])
    if P["we"] is not None:
        _chk(P["we"], torch.bfloat16, "we", P["hidP"] * P["CinP"])
    _chk(P["wd"], torch.float32, "wd", 9 * P["hidP"])
    _chk(P["wp"], torch.bfloat16, "wp", P["CoutP"] * P["hidP"])
    exp_oh = (IH - 1) // P["stride"] + 1
    if (OH, OW) != (exp_oh, (IW - 1) // P["stride"] + 1):
        raise ValueError("fused_ir: output size mismatch")
    _hip_mod().fused_ir(_ptr(x), _ptr(P["we"]), _ptr(P["be"]), _ptr(P["wd"]), _ptr(P["bd"]),
                        _ptr(P["wp"]), _ptr(P["bp"]), _ptr(out), B, IH, IW, P["Cin"], P["CinP"],
                        P["hidP"], P["Cout"], OH, OW, P["stride"], int(P["residual"]), _stream(),
                        P.get("dil", 1), TY, TX, _ptr(P["wd_h"]), _ptr(P["bd_h"]), _ptr(P["wp_h"]),
                        _ptr(trace))
    _dbg('fused_ir')
    return out


def dw_project(hid_in, wd, bd, wp, bp, out, *, B, IH, IW, hid, Cout, OH, OW, stride=1, dil=1,
               res=None):
    """Depthwise 3x3 + ReLU6 fused with the 1x1 projection. wp: [CoutP, hid] bf16."""
    CoutP = (Cout + 15) // 16 * 16
    if hid % 32:
        raise ValueError("dw_project: hid must be a multiple of 32")
    _chk(hid_in, torch.bfloat16, "hid_in", B * IH * IW * hid)
    _chk(wd, torch.float32, "wd", 9 * hid)
    _chk(bd, torch.float32, "bd", hid)
    _chk(wp, torch.bfloat16, "wp", CoutP * hid)
    _chk(bp, torch.float32, "bp", CoutP)
    _chk(out, torch.bfloat16, "out", B * OH * OW * Cout)
    if res is not None:
        _chk(res, torch.bfloat16, "res", B * OH * OW * Cout)
    _hip_mod().dw_project(_ptr(hid_in), _ptr(wd), _ptr(bd), _ptr(wp), _ptr(bp), _ptr(res), _ptr(out),
                          B, IH, IW, hid, Cout, OH, OW, stride, dil, _stream())
    _dbg('dw_project')
    return out


DWP_COUT = (64, 96, 160, 320)  # dw_proj_fused instantiations


def pack_dw_proj(wp: torch.Tensor, wd9: torch.Tensor, bd: torch.Tensor) -> torch.Tensor:
    """Operand of dw_proj_fused (fp16). wp [Cout, hid] projection, wd9 [9, hid]
    depthwise (tap-major), bd [hid]. Per 32-channel hidden chunk c: the projection
    fragments [Cout/16][64 lanes][8], element (n, lane, e) = wp[n*16 + lane%16][c*32 +
    (lane//16)*8 + e], then wd9[:, c*32:(c+1)*32] and bd[c*32:(c+1)*32], zero-padded
    to (Cout/16 + 1) KiB."""
    Cout, hid = wp.shape
    NS, NC = Cout // 16, hid // 32
    frag = wp.float().reshape(NS, 16, NC, 4, 8).permute(2, 0, 3, 1, 4).reshape(NC, NS * 512)
    dw = torch.zeros(NC, 512, dtype=torch.float32, device=wp.device)  # 1 KiB of fp16
    dw[:, :288] = wd9.float().reshape(9, NC, 32).permute(1, 0, 2).reshape(NC, 288)
    dw[:, 288:320] = bd.float().reshape(NC, 32)
    return torch.cat([frag, dw], dim=1).to(torch.float16).contiguous()


def dw_proj_fused(h, wpk, bp, out, *, B, IH, IW, hid, Cout, OH, OW, stride=1, dil=1, res=None,
                  waves=4, rows=0, stages=2, xcd=False):
    """Depthwise 3x3 + ReLU6 + 1x1 projection (+ residual), dw_proj.hip. h [B,IH,IW,hid]
    fp16 (pw_conv out_f16); wpk from ``pack_dw_proj``; bp [Cout] fp32; out bf16.
    ``rows > 0``: row-tile variant (``rows`` output rows per workgroup, halo in LDS,
    a ``stages``-deep LDS ring, ``xcd``: an image's row tiles on one XCD)."""
    if hid % 32 or Cout not in DWP_COUT or waves not in (4, 8):
        raise ValueError(f"dw_proj_fused: unsupported hid={hid} Cout={Cout}")
    if rows and not (1 <= rows <= 255 and stages in (2, 3, 4)):
        raise ValueError("dw_proj_fused: rows 1..255, stages 2..4")
    if rows:
        halo = (rows + 2 * dil) * (OW + 2 * dil)
        lds = stages * ((-(-halo // 16) * 16) * 64 + (Cout // 16 + 1) * 1024)
        if lds > 160 * 1024:
            raise ValueError("dw_proj_fused: row tile too large for LDS at this depth")
    if rows and (stride != 1 or -(-rows * OW // 16) > 16):
        raise ValueError("dw_proj_fused: row tiles need stride 1 and <= 256 pixels")
    if (OH, OW) != ((IH - 1) // stride + 1, (IW - 1) // stride + 1):
        raise ValueError("dw_proj_fused: output size mismatch")
    _chk(h, torch.float16, "h", B * IH * IW * hid)
    _chk(wpk, torch.float16, "wpk", (hid // 32) * (Cout // 16 + 1) * 512)
    _chk(bp, torch.float32, "bp", Cout)
    _chk(out, torch.bfloat16, "out", B * OH * OW * Cout)
    if res is not None:
        _chk(res, torch.bfloat16, "res", B * OH * OW * Cout)
    _hip_mod().dw_proj_fused(_ptr(h), _ptr(wpk), _ptr(bp), _ptr(res), _ptr(out), B, IH, IW, hid,
                             Cout, OH, OW, stride, dil, waves, _stream(),
                             (rows | (stages << 8) | (int(bool(xcd)) << 12)) if rows else 0)
    _dbg('dw_proj_fused')
    return out


def pack_project_padded(wp, bp, Cout, hid, device):
    """Projection weights [Cout, hid] -> zero-padded [CoutP, hid] bf16 + [CoutP] fp32."""
    CoutP = (Cout + 15) // 16 * 16
    w = torch.zeros(CoutP, hid, dtype=torch.float32, device=device)
    w[:Cout] = wp
    b = torch.zeros(CoutP, dtype=torch.float32, device=device)
    b[:Cout] = bp
    return w.to(torch.bfloat16).contiguous(), b


# (Cout/16, CinP/32) shapes the tile kernel is instantiated for (fused_ir.hip);
# blocks without expansion: Cout <= 16 and Cin <= 32
FUSED_TILE_SHAPES = {(4, 2), (6, 2), (6, 3), (10, 3), (10, 5), (20, 5), (4, 1), (2, 1)}
FUSED_TILE_SHAPES_NOEXP = {(1, 1)}


def fused_ir_tile_lds(CinP, stride, dil, TY, TX, expand=True) -> int:
    return int(_hip_mod().fused_ir_tile_lds(CinP, stride, dil, TY, TX, int(expand)))


def pack_fused_ir(we, be, wd, bd, wp, bp, *, Cin, hid, Cout, stride, residual, device,
                  dil=1) -> dict:
    """Zero-pad folded block weights to the fused kernel's layout.

    we: [hid, Cin] (or None when the block has no expansion), wd: [hid, 3, 3],
    wp: [Cout, hid]; biases fp32."""
    r32 = lambda v: (v + 31) // 32 * 32
    CinP = r32(Cin)
    hidP = r32(hid) if we is not None else CinP
    CoutP = (Cout + 15) // 16 * 16
    f32 = dict(dtype=torch.float32, device=device)
    out = dict(Cin=Cin, CinP=CinP, hidP=hidP, Cout=Cout, CoutP=CoutP, stride=stride,
               residual=residual, we=None, dil=dil)
    if we is not None:
        t = torch.zeros(hidP, CinP, **f32)
        t[:hid, :Cin] = we
        out["we"] = t.to(torch.bfloat16).contiguous()
    b = torch.zeros(hidP, **f32)
    if be is not None:
        b[:hid] = be
    out["be"] = b
    t = torch.zeros(9, hidP, **f32)
    t[:, :hid] = wd.reshape(hid, 9).t()
    out["wd"] = t.contiguous()
    b = torch.zeros(hidP, **f32)
    b[:hid] = bd
    out["bd"] = b
    t = torch.zeros(CoutP, hidP, **f32)
    t[:Cout, :hid] = wp
    out["wp"] = t.to(torch.bfloat16).contiguous()
    out["wp_h"] = t.to(torch.float16).contiguous()  # tile kernel: fp16 internals
    out["wd_h"] = out["wd"].to(torch.float16).contiguous()
    out["bd_h"] = out["bd"].to(torch.float16).contiguous()
    b = torch.zeros(CoutP, **f32)
    b[:Cout] = bp
    out["bp"] = b
    return out


def pack_stem_block0(stem, wd, bd, wp, bp, device) -> dict:
    """Weights of the fused stem + block-0 kernel. stem: ConvBNAct (3x3 s2, 3 -> 32);
    wd [32, 3, 3], bd [32], wp [16, 32], bp [16] (BN folded)."""
    w, b = stem.fold()                                   # [32, 3, 3, 3] (RGB in)
    # both ReLU6 as [0, 1] clamps (relu6(v) = 6 clamp(v / 6, 0, 1)): the stem and the
    # depthwise bias are packed / 6 and the projection x 6, so the kernels' clamps fold into
    # the f32 -> f16 conversion and the depthwise's last fma (no min / max instructions)
    ws = torch.zeros(32, 12, 4, dtype=torch.float32)     # K = tap*4 + c: 3 x 16x16x16 MFMA
    ws[:, :9, :3] = w.float().permute(0, 2, 3, 1).reshape(32, 9, 3) / 6.0
    ws = ws.reshape(32, 48)
    f32 = dict(dtype=torch.float32, device=device)
    return dict(
        ws=ws.to(device=device, dtype=torch.bfloat16).contiguous(), bs=(b.float() / 6.0).to(**f32).contiguous(),
        wd_h=wd.reshape(32, 9).t().contiguous().to(device=device, dtype=torch.float16),
        bd_h=(bd.float() / 6.0).to(device=device, dtype=torch.float16).contiguous(),
        wp_h=(wp.float() * 6.0).to(device=device, dtype=torch.float16).contiguous(),
        bp=bp.to(**f32).contiguous(), Cout=int(wp.shape[0]))


def stem_block0(frames, lut_x, lut_y, packed: dict, out, *, H, W, tile=(8, 16)):
    """Fused stem + MobileNetV2 block 0. frames [B, Hc, Wc, 3] u8 BGR; out [B, SH, SW, 16] bf16.
    tile = (TY, TX) output pixels per workgroup, TY*TX <= 256."""
    B, Hc, Wc, _ = frames.shape
    if not (tile[0] >= 1 and 1 <= tile[1] <= 120 and tile[0] * tile[1] <= 256):
        raise ValueError("stem_block0: tile must hold <= 256 pixels")
    _chk(packed["ws"], torch.bfloat16, "ws", 32 * 48)
    SH, SW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    _chk(frames, torch.uint8, "frames", B * Hc * Wc * 3)
    _chk(out, torch.bfloat16, "out", B * SH * SW * packed["Cout"])
    _chk(lut_x, torch.int32, "lut_x", W)
    _chk(lut_y, torch.int32, "lut_y", H)
    P = packed
    _hip_mod().stem_block0(_ptr(frames), _ptr(lut_x), _ptr(lut_y), _ptr(P["ws"]), _ptr(P["bs"]),
                           _ptr(P["wd_h"]), _ptr(P["bd_h"]), _ptr(P["wp_h"]), _ptr(P["bp"]),
                           _ptr(out), B, Hc, Wc, H, W, SH, SW, P["Cout"], tile[0], tile[1],
                           _stream())
    _dbg("stem_block0")
    return out


def stem_band(frames, lut_x, lut_y, packed: dict, out, *, H, W, R=16, nbx=3, one_barrier=True):
    """Row-streaming stem + block 0 (csrc/hip/stem_band.hip): bands of R output rows x
    ceil(SW / nbx) columns; same weights and bit-identical results as ``stem_block0``.
    ``one_barrier``: one workgroup barrier per stem row (double-buffered stem row; False:
    the round-4 two-barrier step)."""
    B, Hc, Wc, _ = frames.shape
    SH, SW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    TW = -(-SW // nbx)
    if R < 1 or nbx < 1 or -(-(TW + 2) // 16) > 8:
        raise ValueError("stem_band: R >= 1 and at most 8 column groups per band")
    _chk(packed["ws"], torch.bfloat16, "ws", 32 * 48)
    _chk(frames, torch.uint8, "frames", B * Hc * Wc * 3)
    _chk(out, torch.bfloat16, "out", B * SH * SW * packed["Cout"])
    _chk(lut_x, torch.int32, "lut_x", W)
    _chk(lut_y, torch.int32, "lut_y", H)
    if packed["Cout"] != 16:
        raise ValueError("stem_band: block 0 projects to 16 channels")
    P = packed
    _hip_mod().stem_band(_ptr(frames), _ptr(lut_x), _ptr(lut_y), _ptr(P["ws"]), _ptr(P["bs"]),
                         _ptr(P["wd_h"]), _ptr(P["bd_h"]), _ptr(P["wp_h"]), _ptr(P["bp"]),
                         _ptr(out), B, Hc, Wc, H, W, SH, SW, R, nbx, _stream(), int(bool(one_barrier)))
    _dbg("stem_band")
    return out


def depthwise3x3(x, w, bias, out, *, B, IH, IW, C, OH, OW, stride=1, dil=1, act="relu6"):
    """x: [B,IH,IW,C] bf16; w: [9, C] fp32; out: [B,OH,OW,C] bf16."""
    _chk(x, torch.bfloat16, "x", B * IH * IW * C)
    _chk(w, torch.float32, "w", 9 * C)
    _chk(bias, torch.float32, "bias", C)
    _chk(out, torch.bfloat16, "out", B * OH * OW * C)
    if C % 8:
        raise ValueError("depthwise3x3: C must be a multiple of 8")
    _hip_mod().depthwise3x3(_ptr(x), _ptr(w), _ptr(bias), _ptr(out), B, IH, IW, C, OH, OW, stride,
                            dil, ACT[act], _stream())
    _dbg('depthwise3x3')
    return out


def stem_conv(frames, lut_x, lut_y, w, bias, out, *, H, W, OH, OW, Cout, k, stride, act,
              out_scale=None):
    """frames: [B,Hc,Wc,3] uint8 BGR; luts int32 [W]/[H]; w: [k*k*3, Cout] fp32."""
    B, Hc, Wc, C3 = frames.shape
    if C3 != 3:
        raise ValueError("frames must be (B, H, W, 3)")
    _chk(frames, torch.uint8, "frames")
    _chk(lut_x, torch.int32, "lut_x", W)
    _chk(lut_y, torch.int32, "lut_y", H)
    _chk(w, torch.float32, "w", k * k * 3 * Cout)
    _chk(bias, torch.float32, "bias", Cout)
    _chk(out, torch.int8 if out_scale else torch.bfloat16, "out", B * OH * OW * Cout)
    _hip_mod().stem_conv(_ptr(frames), _ptr(lut_x), _ptr(lut_y), _ptr(w), _ptr(bias), _ptr(out), B,
                         Hc, Wc, H, W, OH, OW, Cout, k, stride, ACT[act], _stream(),
                         1.0 / out_scale if out_scale else 0.0)
    _dbg('stem_conv')
    return out


def pack_stem_mfma(w: torch.Tensor, k: int, Cout: int) -> torch.Tensor:
    """stem_conv weights [k*k*3, Cout] fp32 -> stem_mfma's bf16 [Cout][ceil(k*k/4)*16]
    (K index = tap * 4 + channel; the 4th channel and the padding taps are zero)."""
    kg = -(-k * k // 4)
    wp = torch.zeros(Cout, kg * 4, 4, dtype=torch.float32, device=w.device)
    wp[:, :k * k, :3] = w.reshape(k * k, 3, Cout).permute(2, 0, 1)
    return wp.reshape(Cout, kg * 16).to(torch.bfloat16).contiguous()


def stem_mfma(frames, lut_x, lut_y, wpk, bias, out, *, H, W, OH, OW, Cout, k, stride, act,
              out_scale=None, tile=(8, 16), per_wave=False):
    """stem_conv on MFMA (TY x TX output tiles); wpk from ``pack_stem_mfma``.
    ``per_wave``: one wave per 16 output channels over the whole tile (7x7 / 64 channels
    only; tiles up to 1024 pixels)."""
    B, Hc, Wc, C3 = frames.shape
    if C3 != 3 or (Cout, k) not in ((64, 7), (32, 3)):
        raise ValueError("stem_mfma: (Cout, k) must be (64, 7) or (32, 3)")
    if per_wave and (Cout, k) != (64, 7):
        raise ValueError("stem_mfma per_wave: (Cout, k) must be (64, 7)")
    ty, tx = tile
    if not (ty >= 1 and tx >= 1 and ty * tx <= (1024 if per_wave else 256) and (per_wave or tx <= 120)):
        raise ValueError("stem_mfma: tile must hold <= 256 pixels (1024 per_wave)")
    if ((ty - 1) * stride + k) * ((tx - 1) * stride + k) * 8 > 64 * 1024:
        raise ValueError("stem_mfma: tile too large")
    _chk(frames, torch.uint8, "frames")
    _chk(lut_x, torch.int32, "lut_x", W)
    _chk(lut_y, torch.int32, "lut_y", H)
    _chk(wpk, torch.bfloat16, "wpk", Cout * (-(-k * k // 4)) * 16)
    _chk(bias, torch.float32, "bias", Cout)
    _chk(out, torch.int8 if out_scale else torch.bfloat16, "out", B * OH * OW * Cout)
    _hip_mod().stem_mfma(_ptr(frames), _ptr(lut_x), _ptr(lut_y), _ptr(wpk), _ptr(bias), _ptr(out), B,
                         Hc, Wc, H, W, OH, OW, Cout, k, stride, ACT[act],
                         1.0 / out_scale if out_scale else 0.0, ty, tx, _stream(), int(per_wave))
    _dbg('stem_mfma')
    return out


# (K fragments of 64, 16-channel subtiles) instantiated by conv_i8.hip's streaming 1x1 kernel
_I8_1X1_INST = ((1, 16), (1, 8), (1, 4), (2, 16), (2, 8), (2, 4), (4, 16), (4, 8), (4, 4), (4, 2),
                (8, 8), (8, 4), (8, 2), (8, 1), (16, 4), (16, 2), (16, 1))


_I8_3X3_INST = ((1, 4), (1, 2), (2, 2), (2, 1),                    # weights in VGPRs (5 / 6)
                (1, 8), (2, 4), (4, 2), (4, 1))                    # + weights in LDS (10 / 11)


def conv_i8_1x1_ok(*, Cin, Cout, k=1, stride=1, ldo=None, co_off=0, int8_out=True, IH=None, OH=None,
                   IW=None, OW=None, **_) -> bool:
    """Whether the streaming variants (5 / 6 / 10 / 11) cover this conv: 1x1 stride 1, or
    3x3 with few enough weight fragments (mirrors conv_i8.hip conv_i8_1x1_ok)."""
    ldo = Cout if ldo is None else ldo
    vec = 16 if int8_out else 8
    if k == 3:
        table, geom = _I8_3X3_INST, True
    else:
        table = _I8_1X1_INST
        geom = k == 1 and (IH is None or OH == (IH - 1) // stride + 1) and (IW is None or OW == (IW - 1) // stride + 1)
    return (geom and Cin % 64 == 0 and Cout % 16 == 0 and ldo % vec == 0 and co_off % vec == 0
            and any(Cin // 64 == cf and (Cout // 16) % ns == 0 for cf, ns in table))


def conv_i8(x, w8, scale, bias, out, *, B, IH, IW, Cin, OH, OW, Cout, k=1, stride=1, dil=1,
            ldo=None, co_off=0, act=None, res=None, res_scale=0.0, img_bias=None,
            out_scale=None, variant=0, perm=None) -> torch.Tensor:
    """int8 NHWC conv. out int8 (out_scale given: v / out_scale rounded) or bf16.
    variant: 0 auto, 1 register-fed, 2/3/4/7/8 LDS-DMA 128x128 / 128x256 / 256x128 / 160x128 /
    96x128 tiles, 12 / 13 = 7 / 2 in n-tile-major block order, 18 / 19 / 20 = 2 / 3 / 4 with
    64-byte K rows per LDS stage (half the LDS: more workgroups per CU),
    5 / 6 / 10 / 11 streaming 1x1 (stride 1; conv_i8_1x1_ok; the widest fitting channel block,
    then narrower ones).
    ``perm`` (LDS-DMA variants only; ``tap_group_perm`` with the variant's tile height): GEMM
    rows -> output pixels, tiles of equal tap validity."""
    if variant not in (0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 13, 18, 19, 20) or (
            variant in (2, 3, 4, 7, 8, 12, 13, 18, 19, 20) and k * k > 16):
        raise ValueError("conv_i8: bad variant")
    Mp = 0
    if perm is not None:
        if variant not in I8_TILE:
            raise ValueError("conv_i8: a row permutation needs an LDS-DMA variant")
        Mp = _check_perm(perm, I8_TILE[variant][0], B * OH * OW, "conv_i8")
    if variant in (5, 6, 10, 11) and not conv_i8_1x1_ok(Cin=Cin, Cout=Cout, k=k, stride=stride, ldo=ldo, co_off=co_off,
                                           int8_out=out_scale is not None):
        raise ValueError("conv_i8: the streaming 1x1 variant does not fit this conv")
    ldo = Cout if ldo is None else ldo
    if Cin % 16:
        raise ValueError("conv_i8: Cin must be a multiple of 16")
    if co_off + Cout > ldo:
        raise ValueError("conv_i8: co_off + Cout > ldo")
    _chk(x, torch.int8, "x", B * IH * IW * Cin)
    _chk(w8, torch.int8, "w", Cout * k * k * Cin)
    _chk(scale, torch.float32, "scale", Cout)
    _chk(bias, torch.float32, "bias", Cout)
    mode = 0 if out_scale is not None else 1
    _chk(out, torch.int8 if mode == 0 else torch.bfloat16, "out", B * OH * OW * ldo)
    if res is not None:
        _chk(res, torch.int8, "res", B * OH * OW * Cout)
    if img_bias is not None:
        _chk(img_bias, torch.float32, "img_bias", B * Cout)
    _hip_mod().conv_i8(_ptr(x), _ptr(w8), _ptr(scale), _ptr(bias), _ptr(img_bias), _ptr(res),
                       float(res_scale), _ptr(out), 1.0 / out_scale if mode == 0 else 1.0, mode, B,
                       IH, IW, Cin, OH, OW, Cout, k, k, stride, dil, ldo, co_off, ACT[act], _stream(),
                       variant, _ptr(perm), Mp)
    _dbg('conv_i8')
    return out


# int8 LDS-DMA tile shapes (BM, BN) by conv_i8 variant
I8_TILE = {2: (128, 128), 3: (128, 256), 4: (256, 128), 7: (160, 128), 8: (96, 128),
           12: (160, 128), 13: (128, 128),  # 12 / 13: 7 / 2 with n-tile-major block order
           18: (128, 128), 19: (128, 256), 20: (256, 128)}  # 2 / 3 / 4 with 64-byte K rows


def _check_perm(perm, BM, M, who):
    _chk(perm, torch.int32, "perm")
    Mp = perm.numel()
    if Mp % BM:
        raise ValueError(f"{who}: perm rows must be a multiple of the tile height {BM}")
    if not getattr(perm, "_ssa_checked", False):
        pc = perm.cpu()
        if pc.min().item() < -1 or pc.max().item() >= M:
            raise ValueError(f"{who}: perm entry out of range")
        perm._ssa_checked = True
    return Mp


def grouped_tile_order_i8(convs: List[dict], variant: int, device=None, xcds: int = 1,
                          by_n: bool = False) -> torch.Tensor:
    """Block -> tile table of ``conv_i8_grouped``: every tile of every conv as
    (group << 24) | tile, heaviest first (work = live taps x 128-channel K chunks): the
    longest-processing-time order of ``grouped_tile_order``, so the light 1x1 and
    border-class tiles fill the tail of the 2-per-CU slots. ``xcds`` > 1: the branch-affine
    XCD assignment of ``grouped_tile_order_branch`` (each XCD's L2 holds one branch's
    weights), LPT inside every XCD."""
    BM, BN = I8_TILE[variant]
    ent, cost, key = [], [], []
    for g, c in enumerate(convs):
        tn = -(-c["Cout"] // BN)
        taps = _tile_taps(c["B"], c["OH"], c["OW"], c.get("k", 1), c.get("dil", 1), BM, c.get("perm"))
        kch = -(-c["Cin"] // 128)
        for tm in range(taps.numel()):
            for n in range(tn):
                ent.append((g << 24) | (tm * tn + n))
                cost.append(int(taps[tm]) * kch)
                key.append((g, n) if by_n else g)
    if xcds > 1:  # branch-affine XCD sets: a 3x3 branch's 4.7 MB of int8 weights (or, by_n, one
        # BN-channel slice of them, 2.4 MB: fits the 4 MiB L2 next to the streamed rows)
        heavy = [k for k in dict.fromkeys(key) if convs[k[0] if by_n else k].get("k", 1) > 1] or list(dict.fromkeys(key))
        return _branch_affine(list(zip(cost, ent, key)), heavy, xcds, device)
    idx = sorted(range(len(ent)), key=lambda i: (-cost[i], i))
    return torch.tensor([ent[i] for i in idx], dtype=torch.int32).to(device).contiguous()


def conv_i8_grouped(convs: List[dict], order: torch.Tensor, variant: int = 7) -> None:
    """Up to 4 independent int8 convs in ONE LDS-DMA grid (the ASPP 1x1 + atrous branches:
    one input, disjoint channel slices of the concat buffer), tiles in the
    ``grouped_tile_order_i8`` table. Each conv is a dict of ``conv_i8``'s arguments (x, w,
    scale, bias, out, B, IH, IW, Cin, OH, OW, Cout, k, stride, dil, ldo, co_off, act, res,
    res_scale, img_bias, out_scale, perm)."""
    if not 1 <= len(convs) <= 4:
        raise ValueError("conv_i8_grouped: 1..4 convs")
    if variant not in (2, 3, 4, 7, 8):
        raise ValueError("conv_i8_grouped: variant must be one of 2, 3, 4, 7, 8")
    BM, BN = I8_TILE[variant]
    tiles, groups = [], []
    for c in convs:
        B, IH, IW, Cin, OH, OW, Cout = (c[n] for n in ("B", "IH", "IW", "Cin", "OH", "OW", "Cout"))
        k, stride, dil = c.get("k", 1), c.get("stride", 1), c.get("dil", 1)
        ldo, co_off = c.get("ldo", Cout), c.get("co_off", 0)
        if Cin % 16 or k * k > 16 or co_off + Cout > ldo:
            raise ValueError("conv_i8_grouped: Cin % 16 == 0, <= 16 taps, co_off + Cout <= ldo")
        out_scale = c.get("out_scale")
        mode = 0 if out_scale is not None else 1
        _chk(c["x"], torch.int8, "x", B * IH * IW * Cin)
        _chk(c["w"], torch.int8, "w", Cout * k * k * Cin)
        _chk(c["scale"], torch.float32, "scale", Cout)
        _chk(c["bias"], torch.float32, "bias", Cout)
        _chk(c["out"], torch.int8 if mode == 0 else torch.bfloat16, "out", B * OH * OW * ldo)
        res, img_bias, perm = c.get("res"), c.get("img_bias"), c.get("perm")
        if res is not None:
            _chk(res, torch.int8, "res", B * OH * OW * Cout)
        if img_bias is not None:
            _chk(img_bias, torch.float32, "img_bias", B * Cout)
        Mp = _check_perm(perm, BM, B * OH * OW, "conv_i8_grouped") if perm is not None else 0
        tiles.append(-(-(Mp or B * OH * OW) // BM) * -(-Cout // BN))
        groups.append((_ptr(c["x"]), _ptr(c["w"]), _ptr(c["scale"]), _ptr(c["bias"]), _ptr(img_bias),
                       _ptr(res), float(c.get("res_scale", 0.0)), _ptr(c["out"]),
                       1.0 / out_scale if mode == 0 else 1.0, mode, B, IH, IW, Cin, OH, OW, Cout, k, k,
                       stride, dil, ldo, co_off, ACT[c.get("act")], _ptr(perm), Mp))
    _chk(order, torch.int32, "order")
    if not getattr(order, "_ssa_checked", False):  # every block maps to a real tile, once
        oc = order.cpu().long()
        g, t = oc >> 24, oc & 0xFFFFFF
        if (g < 0).any() or (g >= len(convs)).any():
            raise ValueError("conv_i8_grouped: order entry out of range")
        if (t >= torch.tensor(tiles)[g]).any() or oc.numel() != sum(tiles) or oc.unique().numel() != oc.numel():
            raise ValueError("conv_i8_grouped: the order table must list every tile once")
        order._ssa_checked = True
    _hip_mod().conv_i8_grouped(groups, _ptr(order), order.numel(), variant, _stream())
    _dbg('conv_i8_grouped')


def maxpool3x3s2_i8(x, out, *, B, IH, IW, C, OH, OW):
    _chk(x, torch.int8, "x", B * IH * IW * C)
    _chk(out, torch.int8, "out", B * OH * OW * C)
    _hip_mod().maxpool3x3s2_i8(_ptr(x), _ptr(out), B, IH, IW, C, OH, OW, _stream())
    _dbg('maxpool_i8')
    return out


def global_avgpool_i8(x, out, ws, *, B, HW, C, scale):
    _chk(x, torch.int8, "x", B * HW * C)
    _chk(out, torch.float32, "out", B * C)
    _chk(ws, torch.float32, "ws", B * 16 * C)
    _hip_mod().global_avgpool_i8(_ptr(x), _ptr(out), _ptr(ws), B, HW, C, float(scale), _stream())
    _dbg('gap_i8')
    return out


def maxpool3x3s2(x, out, *, B, IH, IW, C, OH, OW):
    _chk(x, torch.bfloat16, "x", B * IH * IW * C)
    _chk(out, torch.bfloat16, "out", B * OH * OW * C)
    _hip_mod().maxpool3x3s2(_ptr(x), _ptr(out), B, IH, IW, C, OH, OW, _stream())
    _dbg('maxpool3x3s2')
    return out


def gap_workspace(B, C, device) -> torch.Tensor:
    return torch.empty(int(_hip_mod().gap_workspace_floats(B, C)), dtype=torch.float32, device=device)


def global_avgpool(x, out, *, B, HW, C, ws=None):
    _chk(x, torch.bfloat16, "x", B * HW * C)
    _chk(out, torch.float32, "out", B * C)
    if ws is None:
        ws = gap_workspace(B, C, x.device)
    _chk(ws, torch.float32, "ws", int(_hip_mod().gap_workspace_floats(B, C)))
    _hip_mod().global_avgpool(_ptr(x), _ptr(out), _ptr(ws), B, HW, C, _stream())
    _dbg('global_avgpool')
    return out


def matvec(x, w, bias, out, *, B, N, K, act=None):
    _chk(x, torch.float32, "x", B * K)
    _chk(w, torch.float32, "w", N * K)
    if bias is not None:
        _chk(bias, torch.float32, "bias", N)
    _chk(out, torch.float32, "out", B * N)
    _hip_mod().matvec(_ptr(x), _ptr(w), _ptr(bias), _ptr(out), B, N, K, ACT[act], _stream())
    _dbg('matvec')
    return out


def aspp_pool(x, ws, w1t, b1, w2t, img_bias, *, B, HW, C, N):
    """ASPP image-pooling branch -> per-image projection bias: GAP (two-pass, ws =
    gap_workspace) then relu(w1t^T gap + b1) and w2t^T pooled in one workgroup per image.
    w1t [C, N] and w2t [N, N] are the transposed fp32 weights."""
    _chk(x, torch.bfloat16, "x", B * HW * C)
    _chk(ws, torch.float32, "ws", int(_hip_mod().gap_workspace_floats(B, C)))
    _chk(w1t, torch.float32, "w1t", C * N)
    _chk(b1, torch.float32, "b1", N)
    _chk(w2t, torch.float32, "w2t", N * N)
    _chk(img_bias, torch.float32, "img_bias", B * N)
    _hip_mod().aspp_pool(_ptr(x), _ptr(ws), _ptr(w1t), _ptr(b1), _ptr(w2t), _ptr(img_bias), B, HW, C, N,
                         _stream())
    _dbg('aspp_pool')
    return img_bias


ASPP_HEAD_G = (1, 2, 3, 5, 9)  # 16-pixel groups per workgroup (aspp_head.hip instantiations)


def _frag_pack(w: torch.Tensor, rows: int) -> torch.Tensor:
    """[N, K] -> MFMA A-fragment order [ceil(rows/16)][K/32][64 lanes][8] bf16, element
    (n, k, lane, e) = W[n*16 + lane%16][k*32 + (lane//16)*8 + e] (rows zero-padded)."""
    N, Kd = w.shape
    NS = -(-rows // 16)
    full = torch.zeros(NS * 16, Kd, dtype=torch.float32, device=w.device)
    full[:N] = w.float()
    return (full.reshape(NS, 16, Kd // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
            .to(torch.bfloat16).reshape(-1))


def pack_aspp_head(proj_w: torch.Tensor, proj_b: torch.Tensor, logit_w: torch.Tensor,
                   logit_b: torch.Tensor, device=None) -> dict:
    """ASPP projection [256, K] + logits [ncls, 256] (folded, fp32 or bf16) -> the
    operands of ``aspp_head``: fragment-packed weights, fp32 biases (logits padded to 32)."""
    proj_w = proj_w.reshape(proj_w.shape[0], -1)
    logit_w = logit_w.reshape(logit_w.shape[0], -1)
    N, Kd = proj_w.shape
    ncls = logit_w.shape[0]
    if N != 256 or Kd % 64 or logit_w.shape[1] != 256 or ncls > 32:
        raise ValueError("pack_aspp_head: needs proj [256, K % 64 == 0], logits [<= 32, 256]")
    dev = device or proj_w.device
    bl = torch.zeros(32, dtype=torch.float32)
    bl[:ncls] = logit_b.detach().float().cpu()
    return dict(wp=_frag_pack(proj_w.detach().cpu(), 256).to(dev),
                bp=proj_b.detach().float().contiguous().to(dev),
                wl=_frag_pack(logit_w.detach().cpu(), 32).to(dev), bl=bl.to(dev), K=Kd, ncls=ncls)


def aspp_head_groups(M: int) -> int:
    """Pixel groups per workgroup: the smallest instantiation that keeps the grid within
    one workgroup per CU (256), else the largest."""
    groups = -(-M // 16)
    for g in ASPP_HEAD_G:
        if -(-groups // g) <= 256:
            return g
    return ASPP_HEAD_G[-1]


def aspp_head(cat, packed: dict, out, *, M: int, HW: int, ldo: int, img_bias=None,
              G: Optional[int] = None, waves: int = 8) -> torch.Tensor:
    """Fused ASPP projection (+bias, +per-image bias, ReLU) and logits conv (aspp_head.hip).
    cat: [M, K] bf16; out: [M, ldo] bf16 logits (channels ncls..ldo-1 written as zeros)."""
    K, ncls = packed["K"], packed["ncls"]
    G = aspp_head_groups(M) if G is None else G
    if G not in ASPP_HEAD_G or K != 1024 or ldo % 4 or not ncls <= ldo <= 32 or waves not in (8, 16):
        raise ValueError(f"aspp_head: unsupported G={G} K={K} ldo={ldo}")
    _chk(cat, torch.bfloat16, "cat", M * K)
    _chk(out, torch.bfloat16, "out", M * ldo)
    _chk(packed["wp"], torch.bfloat16, "wp", 256 * K)
    _chk(packed["wl"], torch.bfloat16, "wl", 32 * 256)
    _chk(packed["bp"], torch.float32, "bp", 256)
    _chk(packed["bl"], torch.float32, "bl", 32)
    if img_bias is not None:
        if M % HW:
            raise ValueError("aspp_head: M must be a multiple of HW with img_bias")
        _chk(img_bias, torch.float32, "img_bias", (M // HW) * 256)
    _hip_mod().aspp_head(_ptr(cat), _ptr(packed["wp"]), _ptr(packed["bp"]), _ptr(img_bias),
                         _ptr(packed["wl"]), _ptr(packed["bl"]), _ptr(out), M, K, HW, ncls, ldo, G,
                         _stream(), waves)
    _dbg('aspp_head')
    return out


UPSAMPLE_VARIANTS = {"rows": 3, "rows_tag": 4, "lane": 1, "lane_tag": 2, "direct": 5, "union": 6, "cand": 7}


def upsample_argmax(logits, labels, *, B, h, w, K, ldk, H, W, variant: int = 0):
    """Bilinear (align_corners) upsample of [B, h, w, ldk] logits + per-pixel argmax
    into uint8 [B, H, W] labels. ``variant``: 0 default or a ``UPSAMPLE_VARIANTS`` id."""
    _chk(logits, torch.bfloat16, "logits", B * h * w * ldk)
    _chk(labels, torch.uint8, "labels", B * H * W)
    if K > ldk:
        raise ValueError("K > ldk")
    if not 0 <= variant <= 7:
        raise ValueError(f"bad upsample variant {variant}")
    _hip_mod().upsample_argmax(_ptr(logits), _ptr(labels), B, h, w, K, ldk, H, W, _stream(),
                               variant)
    _dbg('upsample_argmax')
    return labels


def post_workspace_bytes(B, H, W, K, bins) -> int:
    return int(_hip_mod().post_workspace_bytes(B, H, W, K, bins))


def postprocess(labels, palette, ws, records, *, B, H, W, crop_h, crop_w, min_area, K, bins,
                thr=127, accum=0):
    """Device contour statistics (csrc/hip/postprocess.hip). ``accum``: the accumulation
    pass over pixel strips (0) or LDS-staged 32 x 32 tiles (1); identical records."""
    _chk(labels, torch.uint8, "labels", B * H * W)
    _chk(palette, torch.int32, "palette", 256 * 3)
    _chk(ws, torch.uint8, "ws", post_workspace_bytes(B, H, W, K, bins))
    _chk(records, torch.float32, "records", B * (1 + 5 * K))
    if not (0 < crop_h <= H and 0 < crop_w <= W):
        raise ValueError("bad crop")
    _hip_mod().postprocess(_ptr(labels), B, H, W, crop_h, crop_w, _ptr(palette), thr,
                           float(min_area), bins, K, _ptr(ws), _ptr(records), _stream(), int(accum))
    _dbg('postprocess')
    return records


def poison_chip(lds: bool = True, regs: bool = True, pat: int = 0x7FC07FC0) -> None:
    """Debug (scripts/debug_poison.py): fill every CU's LDS and every SIMD's register
    file with a NaN pattern, so the next kernel sees poison wherever it reads on-chip
    state it did not write itself."""
    from .native import hip_debug
    if lds:
        hip_debug().poison_lds(pat, 256 * 8, _stream())
    if regs:
        hip_debug().poison_regs(256 * 4 * 8, _stream())


def copy_to_host(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """src (contiguous CUDA tensor) -> dst (contiguous PINNED host tensor of the same byte
    size), by a kernel on the current stream: unlike a D2H hipMemcpyAsync it never blocks
    the launching thread (profiles/r3_lag_stall.txt). Ordering as for any kernel: the
    host may read dst once an event recorded after this call has completed."""
    if not src.is_cuda or dst.is_cuda or not dst.is_pinned():
        raise ValueError("copy_to_host: CUDA source, pinned host destination")
    if not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("copy_to_host: contiguous tensors required")
    nb = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != nb:
        raise ValueError("copy_to_host: byte sizes differ")
    _hip_mod().copy_to_host(src.data_ptr(), dst.data_ptr(), nb, _stream())
    return dst


def pack_rows(dst: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """dst[r] = [a[r] | b[r]] by one kernel on the current stream. dst: contiguous CUDA
    (rows, wa + wb) 4-byte tensor; a, b: contiguous (rows, w) 4-byte tensors on the device
    or in PINNED host memory (the kernel reads those over the bus: no H2D memcpy)."""
    if not dst.is_cuda:
        raise ValueError("pack_rows: CUDA destination")
    for t in (dst, a, b):
        if t.dim() != 2 or t.element_size() != 4 or not t.is_contiguous():
            raise ValueError("pack_rows: contiguous 2-D tensors of 4-byte elements required")
        if not (t.is_cuda or t.is_pinned()):
            raise ValueError("pack_rows: sources must be device or pinned host memory")
    rows = dst.shape[0]
    if a.shape[0] != rows or b.shape[0] != rows or dst.shape[1] != a.shape[1] + b.shape[1]:
        raise ValueError(f"pack_rows: shapes {tuple(dst.shape)} != [{tuple(a.shape)} | {tuple(b.shape)}]")
    _hip_mod().pack_rows(dst.data_ptr(), a.data_ptr(), a.shape[1], b.data_ptr(), b.shape[1], rows,
                         _stream())
    return dst
