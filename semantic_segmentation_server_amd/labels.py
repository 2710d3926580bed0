"""Label files and class colormaps.

Label-file format parity: the reference parses each line with the regex
``\\s*(\\d+)(.+)`` into ``{int: name.strip()}`` (``sem_seg_server.py:30-34``).
We accept exactly the same files (``assets/pascal_voc_segmentation_labels.txt``
is the reference's ``models/pascal_voc_segmentation_labels.txt``), but skip blank
lines instead of crashing on them (the reference's ``p.match(line)`` returns
``None`` for a blank line and ``.groups()`` raises).

Colormap parity: ``pascal_colormap`` reproduces the bit-interleaved PASCAL VOC
palette built by ``create_pascal_label_colormap`` (``sem_seg_server.py:36-50``).
The table is computed once and cached (the reference rebuilds it for every frame
inside ``label_to_color_image``, ``:70``). On the device the palette is baked into
the mask kernel (``csrc/hip/postprocess.hip``) and never materialised as an RGB
image.
"""
from __future__ import annotations

import functools
import os
import re
from typing import Dict

import numpy as np

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
PASCAL_LABELS = os.path.join(ASSET_DIR, "pascal_voc_segmentation_labels.txt")
CITYSCAPES_LABELS = os.path.join(ASSET_DIR, "cityscapes_labels.txt")

_LINE = re.compile(r"\s*(\d+)(.+)")


def parse_labels(text: str) -> Dict[int, str]:
    """Parse label-file text into ``{class_id: name}``."""
    out: Dict[int, str] = {}
    for line in text.splitlines():
        if not line.strip():
            continue
        m = _LINE.match(line)
        if m is None:
            raise ValueError(f"malformed label line: {line!r}")
        num, name = m.groups()
        out[int(num)] = name.strip()
    return out


def load_labels(path: str = PASCAL_LABELS) -> Dict[int, str]:
    with open(path, "r", encoding="utf-8") as f:
        return parse_labels(f.read())


def label_name(labels: Dict[int, str], idx: int) -> str:
    """Name for a class id.

    The reference uses ``labels.get(idx, 0)`` (``sem_seg_server.py:108``), which
    would put an ``int`` into the proto's ``string label`` field and raise. We
    return the decimal id as a string for unknown classes instead.
    """
    return labels.get(int(idx), str(int(idx)))


@functools.lru_cache(maxsize=None)
def _pascal_colormap_cached() -> np.ndarray:
    # Palette entry for class c: bit k of each channel comes from bit (3*j + ch)
    # of c, where j counts 3-bit groups from the LSB and lands at bit (7 - j).
    idx = np.arange(256, dtype=np.int64)
    cmap = np.zeros((256, 3), dtype=np.int64)
    for j in range(8):
        group = idx >> (3 * j)
        for ch in range(3):
            cmap[:, ch] |= ((group >> ch) & 1) << (7 - j)
    cmap.setflags(write=False)
    return cmap


def pascal_colormap() -> np.ndarray:
    """(256, 3) int64 RGB palette of the PASCAL VOC benchmark."""
    return _pascal_colormap_cached()


def label_to_color_image(label: np.ndarray) -> np.ndarray:
    """Map an (H, W) label map to an (H, W, 3) RGB palette image.

    Same checks as the reference (``sem_seg_server.py:67-73``): rank must be 2 and
    labels must index the 256-entry palette.
    """
    label = np.asarray(label)
    if label.ndim != 2:
        raise ValueError("Expect 2-D input label")
    cmap = pascal_colormap()
    if label.size and int(label.max()) >= len(cmap):
        raise ValueError("label value too large.")
    return cmap[label]


# Fixed-point BGR->gray weights of OpenCV's cvtColor(COLOR_BGR2GRAY) for 8-bit
# data: round(0.114 * 2^14), round(0.587 * 2^14), round(0.299 * 2^14).
GRAY_W_B, GRAY_W_G, GRAY_W_R = 1868, 9617, 4899
GRAY_SHIFT = 14


@functools.lru_cache(maxsize=None)
def pascal_foreground_gray() -> np.ndarray:
    """Gray level of each undiluted class colour as the reference computes it.

    The reference converts an RGB palette image with ``COLOR_BGR2GRAY``
    (``sem_seg_server.py:82``), so the palette's R channel gets the *blue* weight.
    Only classes whose gray level exceeds 127 can ever form a contour
    (``:85``): for PASCAL that is car (7 -> 128) and person (15 -> 135).
    """
    cmap = pascal_colormap()
    g = (cmap[:, 0] * GRAY_W_B + cmap[:, 1] * GRAY_W_G + cmap[:, 2] * GRAY_W_R
         + (1 << (GRAY_SHIFT - 1))) >> GRAY_SHIFT
    g.setflags(write=False)
    return g


def cityscapes_colormap() -> np.ndarray:
    """(256, 3) palette used for the Cityscapes-19 config (train ids 0..18).

    Standard Cityscapes train-id colours; unused entries are black. The
    mask stage applies the same palette -> gray -> threshold rule to it.
    """
    colors = [
        (128, 64, 128), (244, 35, 232), (70, 70, 70), (102, 102, 156), (190, 153, 153),
        (153, 153, 153), (250, 170, 30), (220, 220, 0), (107, 142, 35), (152, 251, 152),
        (70, 130, 180), (220, 20, 60), (255, 0, 0), (0, 0, 142), (0, 0, 70),
        (0, 60, 100), (0, 80, 100), (0, 0, 230), (119, 11, 32),
    ]
    cmap = np.zeros((256, 3), dtype=np.int64)
    cmap[: len(colors)] = np.asarray(colors, dtype=np.int64)
    return cmap


def colormap_for(dataset: str) -> np.ndarray:
    if dataset == "pascal":
        return pascal_colormap()
    if dataset == "cityscapes":
        return cityscapes_colormap()
    raise ValueError(f"unknown dataset {dataset!r}")
