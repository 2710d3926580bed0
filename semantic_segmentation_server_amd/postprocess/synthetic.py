"""Synthetic label maps for post-processing tests and benchmarks.

Random weights almost never produce ``car``/``person`` blobs (the only PASCAL
classes whose palette colour survives the reference's gray > 127 test), so the
post-processing stage is exercised with planted label maps: blocky background
classes plus filled ellipses, rings (holes), nested blobs (a blob inside a hole
inside a blob), blobs cut by the image border and speckle noise.
"""
from __future__ import annotations

import numpy as np

BG_CLASSES = (0, 1, 2, 3, 4, 5, 6, 8, 9, 11, 12, 19, 20)
FG_CLASSES = (7, 15)


def random_label_map(rng: np.random.Generator, h: int, w: int, n_blobs: int = 6,
                     fg=FG_CLASSES, noise: float = 0.002, block: int = 32) -> np.ndarray:
    lab = rng.choice(BG_CLASSES, size=(max(h // block, 1) + 1, max(w // block, 1) + 1))
    lab = np.kron(lab, np.ones((block, block), np.int64))[:h, :w].copy()
    yy, xx = np.mgrid[0:h, 0:w]
    for _ in range(n_blobs):
        cy, cx = rng.uniform(-0.1 * h, 1.1 * h), rng.uniform(-0.1 * w, 1.1 * w)
        ry, rx = rng.uniform(2, max(h / 3, 3)), rng.uniform(2, max(w / 3, 3))
        c = rng.choice(fg)
        e = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2
        kind = rng.integers(0, 3)
        if kind == 0:
            lab[e < 1] = c
        elif kind == 1:
            lab[(e < 1) & (e > 0.35)] = c
        else:
            lab[e < 1] = c
            lab[e < 0.5] = rng.choice([0, 3, 8])
            lab[e < 0.15] = rng.choice(fg)
    m = rng.random((h, w)) < noise
    lab[m] = rng.choice([0, 7, 15], size=int(m.sum()))
    return lab.astype(np.uint8)
