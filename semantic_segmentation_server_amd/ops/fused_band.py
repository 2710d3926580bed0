"""Host side of the row-streaming fused inverted-residual kernel (csrc/hip/fused_ir_band.hip).

The kernel runs one MobileNetV2 inverted residual with Cin <= 32, stride 1 or 2 and
dilation 1 (blocks 1-6 of DeepLabv3-MobileNetV2) over bands of R full-width output rows
(ceil(OW / 16) waves), expanding each input row once into an on-chip fp16
row and accumulating the depthwise per row in registers. This module builds the one
weight blob the kernel copies into LDS, launches it, and re-executes its data flow in
numpy from the packed bytes (CPU tests of the packing without a GPU).

Blob sections (16-byte aligned, offsets returned by ``pack_fused_band``):
  We  [hidP/16][64 lanes][8] bf16  expansion A fragments / 6, lane = kq*16 + r:
      We[hs*16 + r][kq*8 + e] / 6 (Cin zero-padded to 32)
  be  [hidP] fp32                  expansion bias / 6
  wd  [9][hidP] fp16               depthwise weights, tap = ky*3 + kx
  bd  [hidP] fp16                  depthwise bias / 6
  Wp  [Cout/16][hidP/32][64][8] fp16 projection A fragments * 6:
      6 * Wp[n*16 + r][c*32 + kq*8 + e]
The 1/6 and 6 fold the two relu6 into [0, 1] clamps (the clamp bit of the instruction
that produces the value, no separate min / max on the VALU).
  bp  [16*ceil(Cout/16)] fp32      projection bias

Reference parity: the model being executed is the reference's
``deeplabv3_mnv2_pascal_quant_edgetpu.tflite`` (/root/reference/sem_seg_server.py:238,162).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

# (stride, hidP / 16, ceil(Cout / 16), waves = ceil(OW / 16)) instantiated in
# fused_ir_band.hip: blocks 1-6 at 513^2 (output widths 129, 129, 65, 65, 65, 33)
BAND_SHAPES = {(2, 6, 2, 9), (1, 10, 2, 9), (2, 10, 2, 5), (1, 12, 2, 5), (2, 12, 4, 3),
               (2, 6, 2, 5), (1, 10, 2, 5)}  # the last two: blocks 1-2 as two column bands


def band_waves(OW: int, split: int = 1) -> int:
    """Column waves of one band: ceil(OW / 16), or for split = 2 those of ceil(OW / 2)."""
    return -(-(-(-OW // 2) if split == 2 else OW) // 16)


def band_supported(cin: int, hid: int, cout: int, stride: int, dil: int, OW: int,
                   split: int = 1) -> bool:
    """A band spans the full output width OW (ceil(OW / 16) waves of 16 columns), or half
    of it (split = 2)."""
    hidP = -(-hid // 32) * 32
    return (dil == 1 and cin <= 32 and cin % 8 == 0 and stride in (1, 2)
            and (stride, hidP // 16, -(-cout // 16), band_waves(OW, split)) in BAND_SHAPES)


def _al(n: int) -> int:
    return (n + 15) // 16 * 16


def pack_fused_band(we: torch.Tensor, be: torch.Tensor, wd: torch.Tensor, bd: torch.Tensor,
                    wp: torch.Tensor, bp: torch.Tensor, *, Cin: int, hid: int, Cout: int,
                    device=None) -> Dict:
    """Folded block weights -> the kernel's blob. we [hid, Cin], wd [hid, 3, 3] (or
    [hid, 9]), wp [Cout, hid]; biases fp32."""
    hidP = -(-hid // 32) * 32
    NSH, NCH, NS = hidP // 16, hidP // 32, -(-Cout // 16)
    f32 = torch.float32
    # relu6 scale folding (see fused_ir_band.hip): E' = E / 6 and D' = D / 6 make both
    # relu6 [0, 1] clamps; the projection weights take the factor 6 back
    We = torch.zeros(hidP, 32, dtype=f32)
    We[:hid, :Cin] = we.detach().float().cpu().reshape(hid, Cin) / 6.0
    fe = We.reshape(NSH, 16, 4, 8).permute(0, 2, 1, 3).contiguous().to(torch.bfloat16)
    Be = torch.zeros(hidP, dtype=f32)
    Be[:hid] = be.detach().float().cpu() / 6.0
    Wd = torch.zeros(9, hidP, dtype=f32)
    Wd[:, :hid] = wd.detach().float().cpu().reshape(hid, 9).t()
    Bd = torch.zeros(hidP, dtype=f32)
    Bd[:hid] = bd.detach().float().cpu() / 6.0
    Wp = torch.zeros(NS * 16, hidP, dtype=f32)
    Wp[:Cout, :hid] = wp.detach().float().cpu().reshape(Cout, hid) * 6.0
    fp = Wp.reshape(NS, 16, NCH, 4, 8).permute(0, 2, 3, 1, 4).contiguous().to(torch.float16)
    Bp = torch.zeros(NS * 16, dtype=f32)
    Bp[:Cout] = bp.detach().float().cpu()
    parts = [fe.view(torch.uint8).reshape(-1), Be.view(torch.uint8).reshape(-1),
             Wd.to(torch.float16).contiguous().view(torch.uint8).reshape(-1),
             Bd.to(torch.float16).contiguous().view(torch.uint8).reshape(-1),
             fp.view(torch.uint8).reshape(-1), Bp.view(torch.uint8).reshape(-1)]
    offs, o = [], 0
    for p_ in parts:
        offs.append(o)
        o = _al(o + p_.numel())
    blob = torch.zeros(o, dtype=torch.uint8)
    for off, p_ in zip(offs, parts):
        blob[off:off + p_.numel()] = p_
    if device is not None:
        blob = blob.to(device)
    return dict(blob=blob, Cin=Cin, hid=hid, hidP=hidP, Cout=Cout, o_be=offs[1], o_wd=offs[2],
                o_bd=offs[3], o_wp=offs[4], o_bp=offs[5], blob_bytes=o)


def band_lds(packed: Dict, stride: int, OW: int, nslot: int, hs: int = 1, split: int = 1) -> int:
    from .hip_ops import _hip_mod
    return int(_hip_mod().fused_ir_band_lds(stride, packed["hidP"], OW, packed["blob_bytes"], nslot,
                                            hs, packed["Cout"], split))


def fused_ir_band(x: torch.Tensor, packed: Dict, out: torch.Tensor, *, B: int, IH: int, IW: int,
                  stride: int, residual: bool, R: int = 8, nslot: int = 2, hs: int = 1,
                  split: int = 1) -> torch.Tensor:
    """Launch fused_ir_band_kernel. x [B, IH, IW, Cin] bf16 -> out [B, OH, OW, Cout] bf16.
    ``hs = 2``: two waves per 16-column group, each owning half of the hidden channels
    (twice the waves per CU at the same LDS, plus a small partial-sum exchange)."""
    from .hip_ops import _chk, _dbg, _hip_mod, _ptr, _stream
    Cin, Cout = packed["Cin"], packed["Cout"]
    OH, OW = (IH - 1) // stride + 1, (IW - 1) // stride + 1
    if residual and (stride != 1 or Cin != Cout):
        raise ValueError("fused_ir_band: residual needs stride 1 and Cin == Cout")
    if nslot not in (1, 2) or R < 1 or hs not in (1, 2) or split not in (1, 2):
        raise ValueError("fused_ir_band: nslot 1 or 2, R >= 1, hs 1 or 2, split 1 or 2")
    if hs == 2 and band_waves(OW, split) > 8:
        raise ValueError("fused_ir_band: hs 2 needs <= 8 column waves (use split 2)")
    if not band_supported(Cin, packed["hid"], Cout, stride, 1, OW, split):
        raise ValueError("fused_ir_band: no instantiation for this block")
    _chk(x, torch.bfloat16, "x", B * IH * IW * Cin)
    _chk(out, torch.bfloat16, "out", B * OH * OW * Cout)
    _chk(packed["blob"], torch.uint8, "blob", packed["blob_bytes"])
    if band_lds(packed, stride, OW, nslot, hs, split) > 160 * 1024:
        raise ValueError("fused_ir_band: LDS over 160 KiB")
    _hip_mod().fused_ir_band(_ptr(x), _ptr(packed["blob"]), _ptr(out), B, IH, IW, Cin, OH, OW, Cout,
                             packed["hidP"], stride, int(bool(residual)), R, nslot,
                             packed["blob_bytes"], packed["o_be"], packed["o_wd"], packed["o_bd"],
                             packed["o_wp"], packed["o_bp"], _stream(), hs, split)
    _dbg("fused_ir_band")
    return out


# ------------------------------------------------------------------ hidden-sliced variant
# (stride, hidP / 32, ceil(Cout / 16), column groups) instantiated in fused_ir_slice.hip;
# waves per workgroup = column groups x hidden chunks <= 16
SLICE_SHAPES = {(2, 3, 2, 5), (2, 3, 2, 4), (1, 5, 2, 3), (1, 5, 2, 2), (2, 5, 2, 3), (2, 5, 2, 2),
                (1, 6, 2, 2), (2, 6, 4, 2), (1, 6, 2, 1), (2, 6, 4, 1)}


def slice_supported(cin: int, hid: int, cout: int, stride: int, dil: int, nw: int) -> bool:
    hidP = -(-hid // 32) * 32
    return (dil == 1 and cin <= 32 and cin % 8 == 0 and stride in (1, 2)
            and (stride, hidP // 32, -(-cout // 16), nw) in SLICE_SHAPES)


def slice_widths(cin: int, hid: int, cout: int, stride: int, dil: int) -> list:
    """Column-group counts instantiated for this block, widest first."""
    return sorted((nw for nw in range(1, 9) if slice_supported(cin, hid, cout, stride, dil, nw)),
                  reverse=True)


def slice_lds(packed: Dict, stride: int, OW: int, nw: int, one_barrier: bool = False) -> int:
    from .hip_ops import _hip_mod
    return int(_hip_mod().fused_ir_slice_lds(stride, packed["hidP"], OW, packed["Cout"], nw,
                                             bool(one_barrier)))


def fused_ir_slice(x: torch.Tensor, packed: Dict, out: torch.Tensor, *, B: int, IH: int, IW: int,
                   stride: int, residual: bool, R: int = 8, nw: int = 2,
                   one_barrier: bool = False) -> torch.Tensor:
    """Launch fused_ir_slice_kernel (csrc/hip/fused_ir_slice.hip): the band kernel's row
    streaming with waves = nw column groups x hidden chunks of 32, each wave's chunk
    weights held in VGPRs. Same blob as fused_ir_band; bit-identical results.
    ``one_barrier``: one workgroup barrier per input row (E / D rows double-buffered)."""
    from .hip_ops import _chk, _dbg, _hip_mod, _ptr, _stream
    Cin, Cout = packed["Cin"], packed["Cout"]
    OH, OW = (IH - 1) // stride + 1, (IW - 1) // stride + 1
    if residual and (stride != 1 or Cin != Cout):
        raise ValueError("fused_ir_slice: residual needs stride 1 and Cin == Cout")
    if R < 1 or not slice_supported(Cin, packed["hid"], Cout, stride, 1, nw):
        raise ValueError("fused_ir_slice: no instantiation for this block / width")
    _chk(x, torch.bfloat16, "x", B * IH * IW * Cin)
    _chk(out, torch.bfloat16, "out", B * OH * OW * Cout)
    _chk(packed["blob"], torch.uint8, "blob", packed["blob_bytes"])
    if slice_lds(packed, stride, OW, nw, one_barrier) > 160 * 1024:
        raise ValueError("fused_ir_slice: LDS over 160 KiB")
    _hip_mod().fused_ir_slice(_ptr(x), _ptr(packed["blob"]), _ptr(out), B, IH, IW, Cin, OH, OW, Cout,
                              packed["hidP"], stride, int(bool(residual)), R, packed["o_be"],
                              packed["o_wd"], packed["o_bd"], packed["o_wp"], packed["o_bp"], nw,
                              _stream(), int(bool(one_barrier)))
    _dbg("fused_ir_slice")
    return out


# ----------------------------------------------------------------------------- emulation
def emulate_fused_band(x: np.ndarray, packed: Dict, *, stride: int, residual: bool) -> np.ndarray:
    """Numpy re-execution of the kernel's math from the packed blob. x: [B, H, W, Cin]
    float (bf16-representable). Returns [B, OH, OW, Cout] fp32 (before the final bf16
    rounding): fp32 expansion -> fp16 [0, 1]-clamped E / 6; fp16 depthwise accumulated per
    input row (ky outer, kx inner), + bd / 6, [0, 1] clamp; fp32 projection (weights x 6)."""
    blob = packed["blob"].cpu().numpy()
    Cin, Cout, hidP = packed["Cin"], packed["Cout"], packed["hidP"]
    NSH, NCH, NS = hidP // 16, hidP // 32, -(-Cout // 16)
    fe = blob[:NSH * 1024].view(np.uint16).astype(np.uint32) << 16
    We = fe.view(np.float32).reshape(NSH, 4, 16, 8).transpose(0, 2, 1, 3).reshape(hidP, 32)
    be = blob[packed["o_be"]:packed["o_be"] + hidP * 4].view(np.float32)
    wd = blob[packed["o_wd"]:packed["o_wd"] + 18 * hidP].view(np.float16).reshape(9, hidP)
    bd = blob[packed["o_bd"]:packed["o_bd"] + 2 * hidP].view(np.float16)
    fp = blob[packed["o_wp"]:packed["o_wp"] + NS * NCH * 1024].view(np.float16).astype(np.float32)
    Wp = fp.reshape(NS, NCH, 4, 16, 8).transpose(0, 3, 1, 2, 4).reshape(NS * 16, hidP)
    bp = blob[packed["o_bp"]:packed["o_bp"] + NS * 64].view(np.float32)
    B, H, W, _ = x.shape
    OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    xp = np.zeros((B, H, W, 32), np.float32)
    xp[..., :Cin] = x
    E = np.clip((xp @ We.T + be).astype(np.float16), 0, 1)        # E / 6, [B, H, W, hidP]
    Ep = np.zeros((B, H + 2, W + 2, hidP), np.float16)
    Ep[:, 1:-1, 1:-1] = E
    D = np.zeros((B, OH, OW, hidP), np.float16)
    for ky in range(3):
        for kx in range(3):
            v = Ep[:, ky:ky + (OH - 1) * stride + 1:stride, kx:kx + (OW - 1) * stride + 1:stride]
            D = (v * wd[ky * 3 + kx] + D).astype(np.float16)
    D = np.clip((D + bd).astype(np.float16), 0, 1).astype(np.float32)   # relu6(.) / 6
    out = D @ Wp[:Cout].T + bp[:Cout]
    if residual:
        out = out + x[..., :Cout]
    return out
