"""Contour statistics without border following — the algorithm of the GPU path.

The reference traces every border (``cv2.findContours``), then for each contour
rasterises a fill and reduces over it (``sem_seg_server.py:88-122``). That is
serial, O(H*W) per contour, and not GPU-friendly. This module computes the same
numbers from connected components and a local (2x2 "quad") decomposition of the
contour polygons, which is what ``csrc/hip/postprocess.hip`` implements; this numpy
version is the readable specification and the CPU path.

Facts used (all verified against the exact tracer in tests):

* Suzuki-Abe contours of an 8-connected foreground are in 1:1 correspondence with
  (a) foreground 8-components (outer borders) and (b) background 4-components that
  do not touch the image border (hole borders).
* Tree: the parent of a foreground component is the background component of the
  pixel left of its first raster pixel (the image border => top level); the parent
  of a hole is the foreground component left of its first pixel.
* Polygons pass through pixel centres, so they decompose over the unit squares
  ("quads") spanned by 2x2 pixel blocks. All foreground corners of a quad belong
  to one component. Per quad, a foreground component with b corners owns a full
  square if b == 4 and the triangle of its corners if b == 3; a hole with a
  corners owns the full square if a >= 2 and the triangle of its corner and that
  corner's two quad neighbours if a == 1. A contour's polygon area and moments are
  the sum of these pieces over its whole subtree in the border tree. All sums are
  integers (a00 = 2*area, a10 = 6*int x dA, a01 = 6*int y dA), so the final
  ``int(m10/m00)`` matches OpenCV's double arithmetic bit for bit.
* Fill of an outer contour = its component plus everything it encloses; fill of a
  hole contour = the hole's subtree plus the parent's pixels 4-adjacent to it.
* Output order = pre-order of the tree with siblings in reverse discovery order
  (discovery point: first pixel for outer borders, the pixel left of the first
  pixel for holes).
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from .reference import palette_mask_numpy

try:  # scipy is only needed for this CPU path
    from scipy import ndimage as _ndi
except Exception:  # pragma: no cover
    _ndi = None

_ONE_SIXTH = 0.16666666666666666666666666666667

# corner order: 0 TL, 1 TR, 2 BL, 3 BR; triangle of a corner = it + its 2 quad neighbours
_TRI_X = np.array([1, 2, 1, 2])   # sum of x offsets (times 1) of the corner's triangle
_TRI_Y = np.array([1, 1, 2, 2])
_OPP = np.array([3, 2, 1, 0])     # b == 3: triangle of the fg corners = triangle of opposite(missing)


def label_components(mask: np.ndarray):
    """Node id per pixel: raster index + 1 of the component's first pixel, 0 for the
    outside background (every bg component touching the image border)."""
    h, w = mask.shape
    fg = mask.astype(bool)
    fl, nf = _ndi.label(fg, structure=np.ones((3, 3), bool))
    bl, nb = _ndi.label(~fg, structure=np.array([[0, 1, 0], [1, 1, 1], [0, 1, 0]], bool))
    idx = np.arange(h * w, dtype=np.int64).reshape(h, w)
    node = np.zeros((h, w), np.int64)
    if nf:
        froot = np.asarray(_ndi.minimum(idx, fl, index=np.arange(1, nf + 1)), np.int64)
        node[fg] = froot[fl[fg] - 1] + 1
    if nb:
        broot = np.asarray(_ndi.minimum(idx, bl, index=np.arange(1, nb + 1)), np.int64) + 1
        edge = np.zeros((h, w), bool)
        edge[0, :] = edge[-1, :] = edge[:, 0] = edge[:, -1] = True
        outside = np.unique(bl[edge & ~fg])
        broot[outside[outside > 0] - 1] = 0
        node[~fg] = broot[bl[~fg] - 1]
    return node, fg


def quad_stats(node: np.ndarray, fg: np.ndarray):
    """Per-node own (a00, a10, a01) from the quad decomposition."""
    h, w = node.shape
    acc = {}
    if h < 2 or w < 2:
        return acc
    ys, xs = np.mgrid[0:h - 1, 0:w - 1]
    xs = xs.astype(np.int64)
    ys = ys.astype(np.int64)
    cn = [node[:-1, :-1], node[:-1, 1:], node[1:, :-1], node[1:, 1:]]
    cf = [fg[:-1, :-1], fg[:-1, 1:], fg[1:, :-1], fg[1:, 1:]]
    nfg = sum(c.astype(np.int64) for c in cf)

    def add(nodes, a00, a10, a01):
        nodes = nodes.ravel()
        keep = nodes != 0
        if not keep.any():
            return
        nodes = nodes[keep]
        for arr, k in ((a00, 0), (a10, 1), (a01, 2)):
            v = np.broadcast_to(arr, node[:-1, :-1].shape).ravel()[keep]
            uniq, inv = np.unique(nodes, return_inverse=True)
            sums = np.zeros(len(uniq), np.int64)
            np.add.at(sums, inv, v.astype(np.int64))
            for u, sv in zip(uniq.tolist(), sums.tolist()):
                acc.setdefault(u, [0, 0, 0])[k] += sv

    # ---- foreground pieces -------------------------------------------------
    fgnode = np.where(cf[0], cn[0], np.where(cf[1], cn[1], np.where(cf[2], cn[2], cn[3])))
    sq = nfg == 4
    add(np.where(sq, fgnode, 0), 2, 6 * xs + 3, 6 * ys + 3)
    tri = nfg == 3
    missing = np.where(~cf[0], 0, np.where(~cf[1], 1, np.where(~cf[2], 2, 3)))
    opp = _OPP[missing]
    add(np.where(tri, fgnode, 0), 1, 3 * xs + _TRI_X[opp], 3 * ys + _TRI_Y[opp])

    # ---- background pieces (holes; node 0 = outside is dropped by add) ---------
    for k in range(4):
        bgk = ~cf[k]
        same = sum(((~cf[j]) & (cn[j] == cn[k])).astype(np.int64) for j in range(4))
        # first corner (in TL,TR,BL,BR order) of its node within the quad
        first = bgk.copy()
        for j in range(k):
            first &= ~((~cf[j]) & (cn[j] == cn[k]))
        sqk = first & (same >= 2)
        add(np.where(sqk, cn[k], 0), 2, 6 * xs + 3, 6 * ys + 3)
        trk = bgk & (same == 1)
        add(np.where(trk, cn[k], 0), 1, 3 * xs + _TRI_X[k], 3 * ys + _TRI_Y[k])
    return acc


def component_segments(labels_cropped: np.ndarray, min_area: float,
                       palette: Optional[np.ndarray] = None,
                       max_records: Optional[int] = None) -> List[tuple]:
    """Same output as ``reference.segments_exact``:
    [(label, score, area_px, cx, cy, order_key, is_hole)] in contour order.

    ``max_records`` (the device's K record slots): when more contours pass min_area,
    keep the ``max_records`` with the smallest node id (raster index of the discovery
    pixel), the device's deterministic rule (postprocess.hip k_assign)."""
    if _ndi is None:
        raise RuntimeError("scipy is required for the CPU component path")
    lab = np.asarray(labels_cropped, np.uint8)
    h, w = lab.shape
    if h == 0 or w == 0:
        return []
    fgm = palette_mask_numpy(lab, palette) > 0
    node, fg = label_components(fgm)
    nodes = np.unique(node)
    nodes = nodes[nodes != 0]
    if len(nodes) == 0:
        return []
    flat_node = node.ravel()
    is_fg = {int(n): bool(fg.ravel()[n - 1]) for n in nodes}
    parent = {}
    for n in nodes.tolist():
        r = n - 1
        y, x = divmod(r, w)
        parent[n] = int(node[y, x - 1]) if x > 0 else 0
    own = quad_stats(node, fg)
    total = {n: list(own.get(n, [0, 0, 0])) for n in nodes.tolist()}
    depth = {}

    def d(n):
        if n == 0:
            return 0
        if n not in depth:
            depth[n] = 1 + d(parent[n])
        return depth[n]

    for n in sorted(nodes.tolist(), key=d, reverse=True):
        p = parent[n]
        if p != 0:
            t = total[p]
            t[0] += total[n][0]; t[1] += total[n][1]; t[2] += total[n][2]
    cand = [n for n in nodes.tolist() if total[n][0] != 0 and total[n][0] * 0.5 >= min_area]
    if max_records is not None and len(cand) > max_records:
        cand = sorted(cand)[:max_records]
    if not cand:
        return []
    # subtree membership per candidate via ancestor walks of every node
    children = {}
    for n in nodes.tolist():
        children.setdefault(parent[n], []).append(n)

    def subtree(n):
        out, st = [], [n]
        while st:
            m = st.pop()
            out.append(m)
            st.extend(children.get(m, []))
        return out

    segs = []
    for n in cand:
        sel = np.isin(flat_node, np.asarray(subtree(n)))
        if not is_fg[n]:
            hole = (node == n)
            adj = np.zeros_like(hole)
            adj[1:, :] |= hole[:-1, :]; adj[:-1, :] |= hole[1:, :]
            adj[:, 1:] |= hole[:, :-1]; adj[:, :-1] |= hole[:, 1:]
            ring = adj & fg & (node == parent[n])
            sel = sel | ring.ravel()
        vals = lab.ravel()[sel]
        hist = np.bincount(vals, minlength=1)
        best = int(np.argmax(hist))
        score = hist[best] / len(vals)
        a00, a10, a01 = total[n]
        m00 = a00 * 0.5
        m10 = a10 * _ONE_SIXTH
        m01 = a01 * _ONE_SIXTH
        if m00 == 0:
            continue
        key = (n - 1) if is_fg[n] else (n - 2)
        segs.append([n, best, score, m00, int(m10 / m00), int(m01 / m00), key, not is_fg[n]])
    # order: pre-order with siblings by descending discovery key
    cset = {s[0]: s for s in segs}

    def chain(n):
        out = []
        while n != 0:
            out.append(n)
            n = parent[n]
        return out[::-1]

    def keyof(n):
        return (n - 1) if is_fg[n] else (n - 2)

    def sort_key(n):
        return [-keyof(m) for m in chain(n)]

    ordered = sorted(cset.keys(), key=sort_key)
    return [(cset[n][1], cset[n][2], cset[n][3], cset[n][4], cset[n][5], cset[n][6], cset[n][7])
            for n in ordered]
