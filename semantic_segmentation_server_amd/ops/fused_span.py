"""Host side of the fused inverted-residual span kernel (csrc/hip/fused_ir_stream.hip).

The kernel runs one MobileNetV2 inverted residual (expand 1x1 + ReLU6 -> depthwise 3x3
dilated + ReLU6 -> project 1x1 [+ residual]) for the output-stride-16 stage with the
6x-expanded tensor kept on chip. This module builds what it reads:

* ``span_table``: the output map of every image is cut into S raster spans of
  ~H*W/S pixels; per span the table holds the span bounds, the first row of its E
  window and the list of its halo pixels (every in-image pixel within Chebyshev
  distance ``dil`` of an output pixel) as ``(pixel << 12) | window position``.
* ``pack_fused_span``: per 32-channel hidden chunk, one contiguous "chunk image" in
  the byte layout the kernel copies into LDS: expansion MFMA fragments (bf16),
  projection fragments (fp16), depthwise weights/bias (fp16) and expansion bias (fp32).
  Both ReLU6 are folded into a [0, 1] clamp: relu6(v) = 6 * clamp(v / 6, 0, 1), so the
  expansion weights/bias and the depthwise bias are packed / 6 and the projection
  weights x 6. The kernel's clamps are then the ``clamp`` bit of its last depthwise
  ``v_pk_fma_f16`` and of the expansion's ``v_cvt_pk_f16_f32`` (no max/min instructions).
* ``emulate_fused_span``: a numpy re-execution of the kernel's data flow from those
  packed bytes (CPU tests of the packing and table logic without a GPU).

Reference parity: the model being executed is the reference's
``deeplabv3_mnv2_pascal_quant_edgetpu.tflite`` (/root/reference/sem_seg_server.py:238,162).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

HDR = 4          # table header ints: p0, p1, wy0, nh
MAX_GROUPS = 9   # output pixel groups per span (kSOG)
NW = 8           # waves per workgroup
RELU6 = 6.0      # folded ReLU6 bound (see pack_fused_span)


def span_geometry(H: int, W: int, S: int, dil: int):
    """Per span: (p0, p1, wy0, rows, halo [(y, x)])."""
    HW = H * W
    out = []
    for j in range(S):
        p0, p1 = j * HW // S, (j + 1) * HW // S
        y0, y1 = p0 // W, (p1 - 1) // W
        mask = np.zeros((H, W), dtype=bool)
        ys = np.arange(p0, p1) // W
        xs = np.arange(p0, p1) % W
        for dy in range(-dil, dil + 1):
            for dx in range(-dil, dil + 1):
                yy, xx = ys + dy, xs + dx
                ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
                mask[yy[ok], xx[ok]] = True
        hy, hx = np.nonzero(mask)  # row-major
        out.append((p0, p1, y0 - dil, (y1 - y0 + 1) + 2 * dil, list(zip(hy.tolist(), hx.tolist()))))
    return out


def span_table(H: int, W: int, S: int, dil: int, device=None) -> Dict:
    if S < 1 or -(-H * W // S) > MAX_GROUPS * 16:
        raise ValueError(f"span_table: spans of {-(-H * W // S)} px exceed {MAX_GROUPS * 16}")
    if 2 * dil + 1 > 16:
        raise ValueError("span_table: dilation too large")
    WCP = W + 16
    geo = span_geometry(H, W, S, dil)
    WR = max(g[3] for g in geo)
    nh_max = max(len(g[4]) for g in geo)
    HG = -(-nh_max // 16)
    xg = max(2, -(-HG // NW))
    if xg > 3:
        raise ValueError(f"span_table: {HG} halo groups exceed 3 per wave")
    if WR * WCP > 4096 or H * W >= (1 << 19):
        raise ValueError("span_table: window or map too large")
    hstride = HDR + xg * NW * 16
    tab = np.zeros((S, hstride), dtype=np.int32)
    for j, (p0, p1, wy0, _rows, halo) in enumerate(geo):
        tab[j, :HDR] = (p0, p1, wy0, len(halo))
        for i, (y, x) in enumerate(halo):
            tab[j, HDR + i] = ((y * W + x) << 12) | ((y - wy0) * WCP + x + dil)
    t = torch.from_numpy(tab)
    if device is not None:
        t = t.to(device)
    return dict(table=t.contiguous(), H=H, W=W, S=S, dil=dil, WR=WR, WCP=WCP, hstride=hstride,
                xg=xg, nh_max=nh_max, xslots=max(0, HG - 2 * NW))


LAT_XQ = 3       # halo groups per expansion wave of the lattice instantiations (<= 192 px)
LAT_PAD = 3      # lattice window pitch = lattice width + 3 (pad column each side, dummy column)


def lattice_order(H: int, W: int, dil: int):
    """Pixels of an H x W map in "lattice" order: the dil^2 phase classes (y % dil, x % dil)
    one after another, each in raster order. Within a class a dilation-``dil`` 3x3 tap is a
    dilation-1 tap of the class grid, so stacking the classes vertically (one zero row
    between them) gives a virtual image of width ceil(W / dil) on which the depthwise is a
    plain 3x3 and a span's halo is its row band +- 1 row instead of +- dil rows.
    Returns (pix, vy, vx) arrays and the virtual width."""
    pix, vys, vxs = [], [], []
    r = 0
    for py in range(dil):
        for px in range(dil):
            Hc, Wc = -(-(H - py) // dil), -(-(W - px) // dil)
            cy, cx = np.meshgrid(np.arange(Hc), np.arange(Wc), indexing="ij")
            pix.append(((py + cy * dil) * W + px + cx * dil).ravel())
            vys.append((r + cy).ravel())
            vxs.append(cx.ravel())
            r += Hc + 1  # one zero row between classes: no tap crosses it
    return np.concatenate(pix), np.concatenate(vys), np.concatenate(vxs), -(-W // dil)


def lattice_table(H: int, W: int, S: int, dil: int, device=None) -> Dict:
    """Span table over the lattice order (see lattice_order): span j is the j-th of S equal
    runs of that order. Same header and halo list as span_table ((pixel << 12) | window
    position, window = the span's virtual rows +- 1, pitch Wv + 3) plus an output list of
    MAX_GROUPS * 16 entries in the same encoding: the kernel (variant bit 8) takes its
    output pixels and their window positions from it, p0 = 0 and p1 = the span's length.
    At 33 x 33, dilation 2, S = 8: 170 halo px per span at most (raster spans: 272), 1.22x
    the output pixels expanded instead of 1.87x (the VERDICT's halo re-expansion)."""
    if dil < 2:
        raise ValueError("lattice_table: dilation >= 2 (at dilation 1 the lattice is the raster)")
    pix, vy, vx, Wv = lattice_order(H, W, dil)
    n = H * W
    WCP = Wv + LAT_PAD
    spans = []
    for j in range(S):
        a, b = j * n // S, (j + 1) * n // S
        if b - a > MAX_GROUPS * 16:
            raise ValueError(f"lattice_table: spans of {b - a} px exceed {MAX_GROUPS * 16}")
        wy0 = int(vy[a:b].min()) - 1
        rows = int(vy[a:b].max()) - wy0 + 2
        occ = {}
        for k in range(a, b):
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    occ[(int(vy[k]) + dy, int(vx[k]) + dx)] = True
        vmap = {(int(y), int(x)): int(p) for p, y, x in zip(pix, vy, vx)}
        halo = sorted((y, x) for (y, x) in occ if (y, x) in vmap)
        spans.append((a, b, wy0, rows, [(vmap[(y, x)], (y - wy0) * WCP + x + 1) for (y, x) in halo]))
    WR = max(sp[3] for sp in spans)
    nh_max = max(len(sp[4]) for sp in spans)
    HG = -(-nh_max // 16)
    xg = max(2, -(-HG // NW))
    if WR * WCP > 4096 or n >= (1 << 19):
        raise ValueError("lattice_table: window or map too large")
    olist = HDR + xg * NW * 16
    hstride = olist + MAX_GROUPS * 16
    tab = np.zeros((S, hstride), dtype=np.int32)
    for j, (a, b, wy0, _rows, halo) in enumerate(spans):
        tab[j, :HDR] = (0, b - a, wy0, len(halo))
        for i, (p, pos) in enumerate(halo):
            tab[j, HDR + i] = (p << 12) | pos
        for i in range(a, b):
            tab[j, olist + i - a] = (int(pix[i]) << 12) | ((int(vy[i]) - wy0) * WCP + int(vx[i]) + 1)
    t = torch.from_numpy(tab)
    if device is not None:
        t = t.to(device)
    return dict(table=t.contiguous(), H=H, W=W, S=S, dil=dil, WR=WR, WCP=WCP, hstride=hstride,
                xg=xg, nh_max=nh_max, xslots=max(0, HG - 2 * NW), lattice=True, olist=olist)


def chunk_bytes(Cin: int, Cout: int) -> int:
    return (2 * (Cin // 32) + Cout // 16 + 1) * 1024


def pack_fused_span(we: torch.Tensor, be: torch.Tensor, wd: torch.Tensor, bd: torch.Tensor,
                    wp: torch.Tensor, bp: torch.Tensor, *, Cin: int, hid: int, Cout: int,
                    device=None) -> Dict:
    """Folded block weights -> chunk images. we [hid, Cin], wd [hid, 3, 3] (or [hid, 9]),
    wp [Cout, hid]; biases fp32. Requires Cin % 32 == 0 and Cout % 16 == 0."""
    if Cin % 32 or Cout % 16:
        raise ValueError("pack_fused_span: Cin % 32 and Cout % 16 required")
    KS, NS = Cin // 32, Cout // 16
    hidP = -(-hid // 32) * 32
    NC = hidP // 32
    f32 = torch.float32
    We = torch.zeros(hidP, Cin, dtype=f32)
    We[:hid] = we.detach().float().cpu().reshape(hid, Cin)
    Be = torch.zeros(hidP, dtype=f32)
    Be[:hid] = be.detach().float().cpu()
    Wd = torch.zeros(hidP, 9, dtype=f32)
    Wd[:hid] = wd.detach().float().cpu().reshape(hid, 9)
    Bd = torch.zeros(hidP, dtype=f32)
    Bd[:hid] = bd.detach().float().cpu()
    Wp = torch.zeros(Cout, hidP, dtype=f32)
    Wp[:, :hid] = wp.detach().float().cpu().reshape(Cout, hid)
    # ReLU6 as a [0, 1] clamp (module docstring): E' = E / 6, D' = D / 6
    We, Be, Bd, Wp = We / RELU6, Be / RELU6, Bd / RELU6, Wp * RELU6
    # expansion fragments: [c][sub][k][lane = kq*16 + r][e] = We[c*32 + sub*16 + r][k*32 + kq*8 + e]
    fe = We.reshape(NC, 2, 16, KS, 4, 8).permute(0, 1, 3, 4, 2, 5).reshape(NC, -1)
    # projection fragments: [c][n][lane][e] = Wp[n*16 + r][c*32 + kq*8 + e]
    fp = Wp.reshape(NS, 16, NC, 4, 8).permute(2, 0, 3, 1, 4).reshape(NC, -1)
    misc = torch.zeros(NC, 1024, dtype=torch.uint8)
    wdc = Wd.reshape(NC, 32, 9).permute(0, 2, 1).reshape(NC, 288).to(torch.float16)
    misc[:, :576] = wdc.contiguous().view(torch.uint8)
    misc[:, 576:640] = Bd.reshape(NC, 32).to(torch.float16).contiguous().view(torch.uint8)
    misc[:, 640:768] = Be.reshape(NC, 32).contiguous().view(torch.uint8)
    img = torch.cat([fe.to(torch.bfloat16).contiguous().view(torch.uint8),
                     fp.to(torch.float16).contiguous().view(torch.uint8), misc], dim=1)
    assert img.shape[1] == chunk_bytes(Cin, Cout)
    bpp = bp.detach().float().cpu().contiguous()
    out = dict(w=img.contiguous(), bp=bpp, Cin=Cin, hid=hid, hidP=hidP, Cout=Cout)
    if device is not None:
        out["w"] = out["w"].to(device)
        out["bp"] = out["bp"].to(device)
    return out


def fused_ir_stream(x: torch.Tensor, packed: Dict, table: Dict, out: torch.Tensor, *, B: int,
                    residual: bool, trace: Optional[torch.Tensor] = None, variant: int = 0,
                    hsplit: int = 1, part: Optional[torch.Tensor] = None,
                    cnt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Launch fused_ir_stream_kernel (csrc/hip/fused_ir_stream.hip): wave-specialised
    expansion / depthwise+projection waves over an LDS-DMA ring of the packed chunk images. x [B, H, W, Cin] bf16, out [B, H, W, Cout] bf16.
    variant 1: the span's ninth output group runs on the expansion waves (balances the two
    roles: the depthwise+projection waves were the critical path, profiles/r3_stream_trace.txt).
    hsplit > 1: each span's hidden chunks are split over ``hsplit`` workgroups (batch 1 has
    B * S = 16..32 workgroups for 256 CUs and the kernel time is one workgroup's serial chunk
    loop, r4 retune tables); their fp32 partials go to ``part`` [hsplit, B*H*W, Cout] and
    stream_combine sums them (+ bias, residual) into ``out``; with ``cnt`` (int32 [B*S],
    zeroed once: each span's last arriving workgroup resets its word) the span's last
    arriving workgroup does that sum inside the launch instead (no combine kernel)."""
    from .hip_ops import _chk, _dbg, _hip_mod, _ptr, _stream
    H, W = table["H"], table["W"]
    Cin, Cout = packed["Cin"], packed["Cout"]
    if residual and Cin != Cout:
        raise ValueError("fused_ir_stream: residual needs Cin == Cout")
    _chk(x, torch.bfloat16, "x", B * H * W * Cin)
    _chk(out, torch.bfloat16, "out", B * H * W * Cout)
    _chk(packed["w"], torch.uint8, "w", (packed["hidP"] // 32) * chunk_bytes(Cin, Cout))
    _chk(packed["bp"], torch.float32, "bp", Cout)
    _chk(table["table"], torch.int32, "table", table["S"] * table["hstride"])
    if trace is not None:
        _chk(trace, torch.int64, "trace", B * table["S"] * 2 * 64)
    if hsplit > 1:
        if part is None:
            raise ValueError("fused_ir_stream: hsplit > 1 needs a partials buffer")
        _chk(part, torch.float32, "part", hsplit * B * H * W * Cout)
        if cnt is not None:
            _chk(cnt, torch.int32, "cnt", B * table["S"])
    lat = bool(table.get("lattice"))
    if lat and variant not in (0, 1, 2, 4):
        raise ValueError("fused_ir_stream: lattice tables run variants 0, 1, 2 and 4")
    _hip_mod().fused_ir_stream(_ptr(x), _ptr(packed["w"]), _ptr(packed["bp"]), _ptr(table["table"]),
                               _ptr(out), B, H, W, Cin, packed["hidP"], Cout, table["dil"],
                               int(bool(residual)), table["S"], table["WR"], table["WCP"],
                               table["hstride"], table["nh_max"], _stream(),
                               0 if trace is None else _ptr(trace), int(variant) | (8 if lat else 0), int(hsplit),
                               0 if hsplit <= 1 else _ptr(part),
                               0 if (hsplit <= 1 or cnt is None) else _ptr(cnt))
    _dbg("fused_ir_stream")
    if hsplit > 1 and cnt is None:
        M = B * H * W
        _hip_mod().stream_combine(_ptr(part), _ptr(packed["bp"]), _ptr(x) if residual else 0, _ptr(out),
                                  int(hsplit), M, Cout, _stream())
        _dbg("stream_combine")
    return out


STREAM_SHAPES = ((64, 64), (64, 96), (96, 96), (96, 160), (160, 160), (160, 320))


def stream_supported(Cin: int, Cout: int, stride: int, H: int, W: int, S: int, dil: int,
                     lattice: bool = False) -> bool:
    """fused_ir_stream instantiations: the 33-wide maps of the headline, dilation 1 (halo
    <= 256 px) or 2 (<= 320 px), spans <= 144 px, LDS within 160 KiB; lattice tables:
    dilation 2, Cin 160 (blocks 14-16), halo <= 192 px."""
    if stride != 1 or (Cin, Cout) not in STREAM_SHAPES or W != 33 or dil not in (1, 2):
        return False
    if (Cin, Cout) == (160, 320) and dil != 2:
        return False
    if lattice and (dil != 2 or Cin != 160):
        return False
    try:
        t = lattice_table(H, W, S, dil) if lattice else span_table(H, W, S, dil)
    except ValueError:
        return False
    if t["nh_max"] > (LAT_XQ * 64 if lattice else (4 if dil == 1 else 5) * 64):
        return False
    from .hip_ops import _hip_mod
    return int(_hip_mod().fused_ir_stream_lds(Cin, Cout, t["WR"], t["WCP"])) <= 160 * 1024 - (MAX_GROUPS * 16 * 4 if lattice else 64)


# ----------------------------------------------------------------------------- emulation
def _f16(a):
    return np.asarray(a, dtype=np.float16)


def emulate_fused_span(x: np.ndarray, packed: Dict, table: Dict, *, residual: bool) -> np.ndarray:
    """Re-execute the kernel's data flow on the CPU from the packed chunk images and the
    span table. x: [B, H, W, Cin] float (bf16-representable). Returns [B, H, W, Cout] fp32
    (before the final bf16 rounding). Mirrors fused_ir_stream_kernel: fp32 expansion, fp16 E
    clamped to [0, 1] (ReLU6 / 6), fp16 depthwise (one fma chain over the 9 taps from the
    bias, the last fma clamped), fp32 projection accumulation."""
    B, H, W, Cin = x.shape
    Cout, hidP = packed["Cout"], packed["hidP"]
    KS, NS, NC = Cin // 32, Cout // 16, hidP // 32
    img = packed["w"].cpu().numpy().reshape(NC, -1)
    tab = table["table"].cpu().numpy()
    S, WCP, WR, d = table["S"], table["WCP"], table["WR"], table["dil"]
    lat, olist = bool(table.get("lattice")), table.get("olist", 0)
    dt = 1 if lat else d  # tap distance in window coordinates
    bp = packed["bp"].cpu().numpy()
    out = np.zeros((B, H * W, Cout), dtype=np.float32)
    xf = x.reshape(B, H * W, Cin).astype(np.float32)
    for c in range(NC):
        ch = img[c]
        fe = ch[: 2 * KS * 1024].view(np.uint16).astype(np.uint32) << 16
        fe = fe.view(np.float32).reshape(2, KS, 4, 16, 8)          # [sub][k][kq][r][e]
        We = fe.transpose(0, 3, 1, 2, 4).reshape(32, Cin)           # [sub*16 + r][k*32 + kq*8 + e]
        fpj = ch[2 * KS * 1024:(2 * KS + NS) * 1024].view(np.float16).astype(np.float32)
        Wp = fpj.reshape(NS, 4, 16, 8).transpose(0, 2, 1, 3).reshape(Cout, 32)
        misc = ch[(2 * KS + NS) * 1024:]
        wd = misc[:576].view(np.float16).reshape(9, 32)
        bd = misc[576:640].view(np.float16)
        be = misc[640:768].view(np.float32)
        for b in range(B):
            for j in range(S):
                p0, p1, wy0, nh = tab[j, :HDR]
                E = np.zeros((WR * WCP, 32), dtype=np.float16)
                ent = tab[j, HDR:HDR + nh]
                px, pos = ent >> 12, ent & 4095
                e = xf[b, px] @ We.T + be                            # fp32 MFMA
                E[pos] = np.clip(_f16(e), 0, 1)
                if lat:  # output pixels and window centres from the table, dilation-1 taps
                    oe = tab[j, olist:olist + p1]
                    ps, ctr = oe >> 12, oe & 4095
                else:
                    ps = np.arange(p0, p1)
                    ctr = (ps // W - wy0) * WCP + ps % W + d
                s = np.broadcast_to(bd, (len(ps), 32)).astype(np.float16)
                for t in range(9):
                    off = (t // 3 - 1) * dt * WCP + (t % 3 - 1) * dt
                    s = _f16(E[ctr + off] * wd[t] + s)
                D = np.clip(s, 0, 1).astype(np.float32)
                out[b, ps] += D @ Wp.T
    out += bp
    if residual:
        out += xf
    return out.reshape(B, H, W, Cout)
