"""Plain-PyTorch reference implementations of the fused device ops.

These are the numerics oracles for the HIP kernels (tests compare each kernel to
the fp32 op here) and the CPU path of config 1. They are *not* a silent fallback
for the GPU path (see ``ops/native.py``).
"""
from __future__ import annotations

from functools import lru_cache
from typing import Tuple

import numpy as np
import torch
import torch.nn.functional as F


def pil_nearest_index(n_in: int, n_out: int) -> np.ndarray:
    """Source index of each output pixel for PIL ``Image.NEAREST`` resize.

    Pillow's scale-affine nearest path starts at ``0.5 * s`` and accumulates
    ``s = n_in / n_out`` in double precision, flooring each position — verified
    bit-exact against Pillow in ``tests/test_preprocess.py``. (The reference
    resizes with PIL NEAREST, ``sem_seg_server.py:155-156``.)
    """
    s = n_in / n_out
    out = np.empty(n_out, dtype=np.int32)
    x = 0.5 * s
    for i in range(n_out):
        out[i] = int(np.floor(x))
        x += s
    return out


@lru_cache(maxsize=64)
def letterbox_luts(cam_w: int, cam_h: int, W: int, H: int, keep_aspect_ratio: bool = True
                   ) -> Tuple[np.ndarray, np.ndarray, int, int, int, int]:
    """Per model column/row: source column/row in the camera frame, -1 = zero pad.

    Returns (lut_x[W], lut_y[H], resized_w, resized_h, crop_w, crop_h); see
    ``postprocess.reference.letterbox_geometry`` for the geometry.
    """
    from ..postprocess.reference import letterbox_geometry
    rw, rh, cw, ch = letterbox_geometry(cam_w, cam_h, W, H, keep_aspect_ratio)
    lx = np.full(W, -1, np.int32)
    ly = np.full(H, -1, np.int32)
    lx[:rw] = pil_nearest_index(cam_w, rw)
    ly[:rh] = pil_nearest_index(cam_h, rh)
    lx.setflags(write=False)
    ly.setflags(write=False)
    return lx, ly, rw, rh, cw, ch


def preprocess(frames_bgr: torch.Tensor, lut_x, lut_y, out_dtype=torch.float32,
               channels_last: bool = False) -> torch.Tensor:
    """uint8 BGR frames (N, Hc, Wc, 3) -> normalised RGB (N, 3, H, W).

    BGR->RGB (``sem_seg_server.py:151``), NEAREST letterbox resize with zero pad
    bottom/right (``:155-156``), then the model's input quantisation
    ``x / 127.5 - 1`` (padding therefore becomes -1).
    """
    dev = frames_bgr.device
    lx = lut_x.long() if torch.is_tensor(lut_x) else torch.as_tensor(np.array(lut_x), device=dev, dtype=torch.long)
    ly = lut_y.long() if torch.is_tensor(lut_y) else torch.as_tensor(np.array(lut_y), device=dev, dtype=torch.long)
    vx, vy = lx >= 0, ly >= 0
    g = frames_bgr[:, ly.clamp(min=0)][:, :, lx.clamp(min=0)]          # N,H,W,3
    g = g * (vy[None, :, None, None] & vx[None, None, :, None])
    rgb = g.flip(-1).to(torch.float32) * (1.0 / 127.5) - 1.0
    out = rgb.permute(0, 3, 1, 2)
    out = out.contiguous(memory_format=torch.channels_last) if channels_last else out.contiguous()
    return out.to(out_dtype)


def upsample_argmax(logits: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """(N, K, h, w) logits -> (N, H, W) uint8 labels: bilinear align_corners=True
    then argmax over K (first max wins, as ``tf.argmax``/``np.argmax``)."""
    up = F.interpolate(logits.float(), size=(H, W), mode="bilinear", align_corners=True)
    return up.argmax(1).to(torch.uint8)


def decisive_agreement(got: torch.Tensor, ref: torch.Tensor, k: float = 4.0) -> Tuple[float, float]:
    """Argmax agreement of ``got`` with ``ref`` (both (N, K, h, w) logits) on the pixels
    whose ``ref`` decision is not a near-tie at the measured error: top-1 minus top-2
    margin > ``k`` x the RMS of ``got - ref``. Returns (agreement, fraction of pixels
    tested). With random-init weights most logits sit within a few bf16 ulps of each
    other, so the plain argmax agreement of any bf16 run (stock PyTorch included: 0.77 /
    0.90 on the same frame in two processes, MIOpen solver choice) is noise; a decision
    with a margin of several error-sigmas must not flip."""
    got, ref = got.float(), ref.float()
    sigma = (got - ref).pow(2).mean().sqrt()
    top2 = ref.topk(2, dim=1).values
    mask = (top2[:, 0] - top2[:, 1]) > k * sigma
    frac = mask.float().mean().item()
    if not bool(mask.any()):
        # nothing decisive: no evidence either way (callers assert a minimum ``frac``)
        return float("nan"), 0.0
    agree = (got.argmax(1) == ref.argmax(1))[mask].float().mean().item()
    return agree, frac
