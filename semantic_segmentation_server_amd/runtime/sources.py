"""Frame sources.

Reference: a single ``cv2.VideoCapture(camera_idx)`` read in the producer loop
(``sem_seg_server.py:144-148``) and probed once at startup for its native
resolution (``:268-270``); end of stream stops the server. OpenCV is not available
here, so:

* ``SyntheticSource`` — deterministic BGR frames (moving coloured shapes plus
  noise) at a given camera resolution; the benchmark source.
* ``FileSource``     — replays ``.npy`` (N, H, W, 3) uint8 stacks or a directory
  of images readable by Pillow.
* ``V4L2Source``     — a V4L2 camera through the native capture in ``_host``
  (``csrc/host/v4l2.cpp``: mmap streaming, YUYV/UYVY -> BGR in C++), no OpenCV;
  ``SSA_CAPTURE=cv2`` selects ``cv2.VideoCapture`` where OpenCV is installed.

Every source yields ``Frame`` objects and exposes ``resolution`` (w, h). Sources
are iterators; ``read_batch(n)`` returns a pinned host batch for the engine.
"""
from __future__ import annotations

import glob
import itertools
import os
import time
from dataclasses import dataclass
from typing import Iterator, List, Optional, Tuple

import numpy as np


@dataclass
class Frame:
    image: np.ndarray      # (H, W, 3) uint8 BGR
    frame_id: int
    stream: int
    ts: float


class FrameSource:
    resolution: Tuple[int, int] = (0, 0)
    stream: int = 0

    def __iter__(self) -> Iterator[Frame]:
        return self

    def __next__(self) -> Frame:  # pragma: no cover
        raise NotImplementedError

    def read_batch(self, n: int) -> Tuple[np.ndarray, List[int], List[float]]:
        frames = list(itertools.islice(self, n))
        if not frames:
            raise StopIteration
        imgs = np.stack([f.image for f in frames])
        return imgs, [f.frame_id for f in frames], [f.ts for f in frames]

    def read_batch_into(self, out: np.ndarray) -> Tuple[int, List[int], List[float]]:
        """Fill ``out`` (n, H, W, 3) in place (the feeder's pinned ring slot); returns
        (frames read, ids, ts). Raises StopIteration when no frame is left."""
        ids, ts = [], []
        for i in range(out.shape[0]):
            try:
                f = next(self)
            except StopIteration:
                if i == 0:
                    raise
                break
            out[i] = f.image
            ids.append(f.frame_id)
            ts.append(f.ts)
        return len(ids), ids, ts

    def close(self) -> None:
        pass


class SyntheticSource(FrameSource):
    """Deterministic synthetic camera.

    Frames are generated from a small pool (``pool``) of pre-rendered images so
    that producing a frame costs a copy, not a render — the source must not be the
    bottleneck of a throughput benchmark.
    """

    def __init__(self, width: int = 640, height: int = 480, stream: int = 0, seed: int = 0,
                 pool: int = 8, limit: Optional[int] = None, fps: Optional[float] = None):
        self.resolution = (int(width), int(height))
        self.stream = stream
        self.limit = limit
        self.fps = fps
        rng = np.random.default_rng(seed + 7919 * stream)
        self.pool = np.stack([self._render(rng, i) for i in range(max(1, pool))])
        self._i = 0
        self._t0 = time.time()

    def _render(self, rng, i) -> np.ndarray:
        w, h = self.resolution
        yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
        img = np.zeros((h, w, 3), np.float32)
        img += rng.uniform(0, 80, 3)
        for _ in range(6):
            cx, cy = rng.uniform(0, w), rng.uniform(0, h)
            rx, ry = rng.uniform(w / 16, w / 3), rng.uniform(h / 16, h / 3)
            m = ((xx - cx) / rx) ** 2 + ((yy - cy) / ry) ** 2 < 1
            img[m] = rng.uniform(0, 255, 3)
        img += rng.normal(0, 8, img.shape)
        return np.clip(img, 0, 255).astype(np.uint8)

    def __next__(self) -> Frame:
        if self.limit is not None and self._i >= self.limit:
            raise StopIteration
        if self.fps:
            target = self._t0 + self._i / self.fps
            dt = target - time.time()
            if dt > 0:
                time.sleep(dt)
        f = Frame(self.pool[self._i % len(self.pool)], self._i, self.stream, time.time())
        self._i += 1
        return f

    def read_batch(self, n: int):
        if self.limit is not None:
            n = min(n, self.limit - self._i)
            if n <= 0:
                raise StopIteration
        idx = (np.arange(self._i, self._i + n) % len(self.pool))
        ids = list(range(self._i, self._i + n))
        self._i += n
        now = time.time()
        return self.pool[idx], ids, [now] * n

    def advance(self, n: int):
        """Consume ``n`` frames without copying pixels (the feeder's replay of a ring
        slot that already holds pool frames)."""
        if self.limit is not None:
            n = min(n, self.limit - self._i)
            if n <= 0:
                raise StopIteration
        ids = list(range(self._i, self._i + n))
        self._i += n
        return n, ids, [time.time()] * n

    def read_batch_into(self, out: np.ndarray):
        n = out.shape[0]
        if self.limit is not None:
            n = min(n, self.limit - self._i)
            if n <= 0:
                raise StopIteration
        if self.fps:  # paced like __next__: the batch is ready when its last frame is
            dt = self._t0 + (self._i + n - 1) / self.fps - time.time()
            if dt > 0:
                time.sleep(dt)
        idx = np.arange(self._i, self._i + n) % len(self.pool)
        np.take(self.pool, idx, axis=0, out=out[:n])
        ids = list(range(self._i, self._i + n))
        self._i += n
        return n, ids, [time.time()] * n


class FileSource(FrameSource):
    def __init__(self, path: str, stream: int = 0, loop: bool = False):
        self.stream = stream
        self.loop = loop
        if path.endswith(".npy"):
            self.frames = np.load(path, mmap_mode="r", allow_pickle=False)
        else:
            from PIL import Image
            files = sorted(glob.glob(os.path.join(path, "*")))
            imgs = [np.asarray(Image.open(f).convert("RGB"))[..., ::-1] for f in files]
            self.frames = np.stack(imgs)
        if self.frames.ndim != 4 or self.frames.shape[-1] != 3:
            raise ValueError("expected (N, H, W, 3) frames")
        self.resolution = (int(self.frames.shape[2]), int(self.frames.shape[1]))
        self._i = 0

    def __next__(self) -> Frame:
        if self._i >= len(self.frames):
            if not self.loop:
                raise StopIteration
            self._i = 0
        f = Frame(np.asarray(self.frames[self._i]), self._i, self.stream, time.time())
        self._i += 1
        return f


class V4L2Source(FrameSource):
    """A V4L2 camera (reference: ``cv2.VideoCapture(camera_idx)``, sem_seg_server.py:144-148,
    probed once for its native resolution at :268-270). ``camera_idx`` is the N of
    ``/dev/videoN``; the driver picks the nearest size to ``width`` x ``height``."""

    def __init__(self, camera_idx: int, stream: int = 0, width: int = 640, height: int = 480,
                 timeout_ms: int = 2000, device: Optional[str] = None):
        self.stream = stream
        self.timeout_ms = int(timeout_ms)
        self._i = 0
        self._cv = None
        self.cap = None
        if os.environ.get("SSA_CAPTURE", "native") == "cv2":  # pragma: no cover - needs cv2
            import cv2
            self._cv = cv2.VideoCapture(camera_idx)
            self.resolution = (int(self._cv.get(cv2.CAP_PROP_FRAME_WIDTH)),
                               int(self._cv.get(cv2.CAP_PROP_FRAME_HEIGHT)))
            return
        from ..ops.native import host
        self.cap = host().V4L2Capture(device or f"/dev/video{int(camera_idx)}", int(width), int(height))
        self.resolution = (int(self.cap.width), int(self.cap.height))

    def _read(self, out: np.ndarray) -> bool:
        if self._cv is not None:  # pragma: no cover
            ok, img = self._cv.read()
            if ok:
                out[...] = img
            return bool(ok)
        ok, _seq, _ts = self.cap.read_into(out, self.timeout_ms)
        return bool(ok)

    def __next__(self) -> Frame:
        w, h = self.resolution
        img = np.empty((h, w, 3), np.uint8)
        if not self._read(img):
            raise StopIteration  # end of stream / camera gone: the producer stops (:146-148)
        f = Frame(img, self._i, self.stream, time.time())
        self._i += 1
        return f

    def read_batch_into(self, out: np.ndarray):
        """Frames straight into the feeder's pinned ring slot (no intermediate copy)."""
        ids, ts = [], []
        for i in range(out.shape[0]):
            if not self._read(out[i]):
                if i == 0:
                    raise StopIteration
                break
            ids.append(self._i)
            ts.append(time.time())
            self._i += 1
        return len(ids), ids, ts

    def close(self):
        if self._cv is not None:  # pragma: no cover
            self._cv.release()
        if self.cap is not None:
            self.cap.close()


def probe_resolution(kind: str, camera_idx: int = 1, width: int = 640, height: int = 480,
                     path: Optional[str] = None) -> Tuple[int, int]:
    """Native resolution of a source (reference probes the camera once, ``:268-270``)."""
    if kind == "synthetic":
        return (width, height)
    if kind == "file":
        return FileSource(path).resolution
    if kind == "camera":
        src = V4L2Source(camera_idx, width=width, height=height)
        res = src.resolution
        src.close()
        return res
    raise ValueError(kind)


def make_source(kind: str, stream: int = 0, camera_idx: int = 1, width: int = 640,
                height: int = 480, path: Optional[str] = None, limit: Optional[int] = None,
                fps: Optional[float] = None, seed: int = 0) -> FrameSource:
    if kind == "synthetic":
        return SyntheticSource(width, height, stream, seed=seed, limit=limit, fps=fps)
    if kind == "file":
        return FileSource(path, stream, loop=limit is None)
    if kind == "camera":
        return V4L2Source(camera_idx + stream, stream, width=width, height=height)
    raise ValueError(kind)
