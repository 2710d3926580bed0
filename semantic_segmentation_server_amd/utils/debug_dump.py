"""Annotated debug frames (``--debug_dump DIR --debug_every N``).

The reference carries this as dead code inside a string literal
(``sem_seg_server.py:196-205``: drawContours on the resized frame, a circle at
each centroid, ``putText`` of the label, ``imshow``). Here it is a working,
headless writer: the letterboxed camera frame, the class colours blended over it,
every contour ``findContours`` would return (from the exact host tracer) and,
for each reported segment, its centroid and ``label score``, saved as PNG.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np

from ..postprocess import reference as PR


def render(frame_bgr: np.ndarray, label_map: np.ndarray, crop_w: int, crop_h: int,
           palette: np.ndarray, names: Dict[int, str], min_area: float, alpha: float = 0.45):
    """-> PIL.Image (RGB) of the model-space valid region (crop_w x crop_h)."""
    from PIL import Image, ImageDraw

    Hc, Wc = frame_bgr.shape[:2]
    H, W = label_map.shape
    # nearest resize of the camera frame into the letterboxed region (same index map as K1)
    from ..ops.reference_ops import letterbox_luts
    lx, ly, *_ = letterbox_luts(Wc, Hc, W, H, True)
    rgb = frame_bgr[..., ::-1]
    img = np.zeros((H, W, 3), np.uint8)
    vy, vx = ly >= 0, lx >= 0
    img[np.ix_(vy, vx)] = rgb[np.ix_(ly[vy], lx[vx])]
    img = img[:crop_h, :crop_w]
    lab = np.ascontiguousarray(label_map[:crop_h, :crop_w], dtype=np.uint8)
    pal = np.asarray(palette, np.int64).reshape(256, 3)
    color = pal[lab].astype(np.float32)
    out = (img.astype(np.float32) * (1 - alpha) + color * alpha).clip(0, 255).astype(np.uint8)
    im = Image.fromarray(out, "RGB")
    dr = ImageDraw.Draw(im)
    host = PR.host_module()
    mask = host.palette_mask(lab, PR.palette_int32(palette), 127)
    for c in host.find_contours(mask):
        pts = c["points"]
        if len(pts) >= 2:
            xy = [tuple(map(int, p)) for p in pts] + [tuple(map(int, pts[0]))]
            dr.line(xy, fill=(0, 255, 0), width=1)
    for lab_id, score, area, cx, cy, _, _ in PR.segments_exact(lab, min_area, palette):
        r = 3
        dr.ellipse((cx - r, cy - r, cx + r, cy + r), outline=(255, 0, 0), width=2)
        dr.text((cx + 5, cy - 5), f"{names.get(int(lab_id), str(lab_id))} {score:.2f}",
                fill=(255, 255, 255))
    return im


class DebugDumper:
    def __init__(self, out_dir: Optional[str], every: int, palette, names, min_area: float):
        self.out_dir = out_dir
        self.every = int(every)
        self.palette, self.names, self.min_area = palette, names, float(min_area)
        self.n = 0
        if self.enabled:
            os.makedirs(out_dir, exist_ok=True)

    @property
    def enabled(self) -> bool:
        return bool(self.out_dir) and self.every > 0

    def want(self) -> bool:
        """Call once per frame batch; True when this batch's first frame is dumped."""
        if not self.enabled:
            return False
        hit = self.n % self.every == 0
        self.n += 1
        return hit

    def dump(self, frame_bgr, label_map, crop_w, crop_h, stream: int, frame_id: int) -> str:
        path = os.path.join(self.out_dir, f"s{stream:03d}_f{frame_id:08d}.png")
        render(frame_bgr, label_map, crop_w, crop_h, self.palette, self.names,
               self.min_area).save(path)
        return path
