"""Reference (exact) post-processing of a label map — the parity oracle.

Implements SURVEY.md §2.3 for one frame, mirroring the reference producer body
(``sem_seg_server.py:163-195``):

1. crop the padded model output to the letterboxed region (``:164-167``);
2. colourise with the palette, 3x3 box blur, BGR2GRAY (on RGB data), ``> 127``
   (``get_segment_contours``, ``:77-90``);
3. ``findContours(RETR_TREE, CHAIN_APPROX_SIMPLE)``;
4. per contour: polygon area, reject ``< min_area`` (``:93-95``); fill, majority
   label and its fraction (``:98-111``); polygon moments, skip ``m00 == 0``,
   truncated centroid (``:115-122``);
5. normalise by the *model input* W, H and clamp to 1 (``:183-192``).

Steps 2-4 run in the host C++ module (``_host.segments``): an exact Suzuki-Abe
tracer written from the paper (OpenCV is not installable here). The records come
out in contour order, i.e. the order the reference ``appendleft``s them.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..labels import pascal_colormap
from ..runtime.results import RECORD_DTYPE


def host_module():
    from ..ops import native
    return native.host()


def letterbox_geometry(cam_w: int, cam_h: int, W: int, H: int,
                       keep_aspect_ratio: bool = True) -> Tuple[int, int, int, int]:
    """Resized size and crop of the model-space valid region.

    Mirrors edgetpu ``image_processing.resampling_with_original_ratio`` [EXT]
    as used at ``sem_seg_server.py:154-167``: scale by
    ``min(W / cam_w, H / cam_h)``, truncate the resized size to int, zero-pad
    bottom/right; the server then crops ``int(W * ratio_w) x int(H * ratio_h)``.

    Returns (resized_w, resized_h, crop_w, crop_h).
    """
    if not keep_aspect_ratio:
        return W, H, W, H
    r = min(W / cam_w, H / cam_h)
    rw, rh = int(cam_w * r), int(cam_h * r)
    ratio_w, ratio_h = rw / W, rh / H
    return rw, rh, int(W * ratio_w), int(H * ratio_h)


def palette_int32(palette: Optional[np.ndarray] = None) -> np.ndarray:
    p = pascal_colormap() if palette is None else palette
    return np.ascontiguousarray(p, dtype=np.int32).reshape(256, 3)


def segments_exact(labels_cropped: np.ndarray, min_area: float,
                   palette: Optional[np.ndarray] = None) -> List[tuple]:
    """[(label, score, area_px, cx, cy, contour_idx, is_hole)] in contour order."""
    lab = np.ascontiguousarray(labels_cropped, dtype=np.uint8)
    return host_module().segments(lab, palette_int32(palette), float(min_area))


def frame_records(label_map: np.ndarray, crop_w: int, crop_h: int, min_area_ratio: float,
                  palette: Optional[np.ndarray] = None, stream: int = 0, frame: int = 0,
                  ts: float = 0.0) -> np.ndarray:
    """Records of one model-resolution label map, in push order."""
    H, W = label_map.shape
    min_area = min_area_ratio * H * W
    segs = segments_exact(label_map[:crop_h, :crop_w], min_area, palette)
    out = np.zeros(len(segs), dtype=RECORD_DTYPE)
    for i, (lab, score, area, cx, cy, _, _) in enumerate(segs):
        out[i] = (lab, score, min(1.0, area / (W * H)), min(1.0, cx / W), min(1.0, cy / H),
                  stream, frame, ts)
    return out


def palette_mask_numpy(labels: np.ndarray, palette: Optional[np.ndarray] = None,
                       thr: int = 127) -> np.ndarray:
    """Vectorised numpy version of the mask stage (same integer arithmetic)."""
    pal = palette_int32(palette).astype(np.int64)
    rgb = pal[labels.astype(np.int64)]
    pad = np.pad(rgb, ((1, 1), (1, 1), (0, 0)), mode="reflect")  # == REFLECT_101
    h, w = labels.shape
    s = np.zeros((h, w, 3), np.int64)
    for dy in range(3):
        for dx in range(3):
            s += pad[dy:dy + h, dx:dx + w]
    c = (s * 2 + 9) // 18
    g = (c[..., 0] * 1868 + c[..., 1] * 9617 + c[..., 2] * 4899 + 8192) >> 14
    return np.where(g > thr, 255, 0).astype(np.uint8)
