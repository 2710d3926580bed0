"""Frame feeder: camera/file/synthetic sources -> a ring of preallocated pinned batches.

Reference: the producer reads one camera frame at a time on the inference thread
(``cap.read()``, ``/root/reference/sem_seg_server.py:146-148``), converts and resizes
it there (``:150-161``) and only then runs the Edge TPU -- capture and inference are
serialised. Here a ``BatchFeeder`` thread assembles each step's batch (round-robin
over the streams, ``batch`` frames) directly into one of ``ring`` page-locked host
buffers allocated once, so the serving loop only issues the async H2D of a ready
buffer: no per-step pinned allocation, no copy on the inference thread, and capture
overlaps the GPU step.

A slot is handed to the consumer with ``get()`` and returned with ``release()`` once
its H2D copy has completed (the consumer checks the copy's event); the feeder blocks
when every slot is in use, so a slow consumer throttles capture instead of queueing
frames without bound.

Synthetic sources serve frames from a fixed pool of pre-rendered images, so after each
ring slot has been filled once (``replay``) a refill only advances the frame ids and
timestamps: a benchmark source must not turn the serving loop into a 30 MB-per-step
host memcpy benchmark (``bench.py`` likewise replays two pinned batches).
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from .sources import FrameSource

log = logging.getLogger(__name__)


@dataclass
class Batch:
    slot: int
    frames: torch.Tensor          # (n, H, W, 3) uint8, pinned when CUDA is available
    ids: List[int] = field(default_factory=list)
    ts: List[float] = field(default_factory=list)
    streams: List[int] = field(default_factory=list)


def split_batch(batch: int, nsrc: int) -> List[int]:
    """Round-robin share of ``batch`` frames over ``nsrc`` streams."""
    per = [batch // nsrc] * nsrc
    for i in range(batch % nsrc):
        per[i] += 1
    return per


class BatchFeeder(threading.Thread):
    _EOS = object()

    def __init__(self, sources: Sequence[FrameSource], batch: int, ring: int = 4,
                 pin: Optional[bool] = None, retry_limit: int = 10, metrics=None):
        super().__init__(name="feeder", daemon=True)
        if not sources:
            raise ValueError("BatchFeeder needs at least one source")
        self.sources = list(sources)
        self.batch = int(batch)
        w, h = self.sources[0].resolution
        if any(s.resolution != (w, h) for s in self.sources):
            raise ValueError("all streams of one feeder must share a resolution")
        self.shape = (self.batch, h, w, 3)
        pin = torch.cuda.is_available() if pin is None else pin
        self.bufs = [torch.empty(self.shape, dtype=torch.uint8, pin_memory=pin) for _ in range(ring)]
        self._free: "queue.Queue[int]" = queue.Queue()
        for i in range(ring):
            self._free.put(i)
        self._ready: "queue.Queue" = queue.Queue()
        self._stop = threading.Event()
        self.retry_limit = retry_limit
        self.metrics = metrics
        self.error: Optional[BaseException] = None
        self.batches = 0
        from .sources import SyntheticSource
        self.replay = all(isinstance(s, SyntheticSource) and s.fps is None for s in self.sources)
        self._filled = [False] * ring

    # --------------------------------------------------------------- producer side
    def _fill(self, slot: int) -> Batch:
        arr = self.bufs[slot].numpy()
        b = Batch(slot, self.bufs[slot])
        off = 0
        for src, n in zip(self.sources, split_batch(self.batch, len(self.sources))):
            if n == 0:
                continue
            if self.replay and self._filled[slot]:
                got, ids, ts = src.advance(n)
            else:
                got, ids, ts = src.read_batch_into(arr[off:off + n])
            if got < n:  # short read at end of stream: repeat the last frame
                arr[off + got:off + n] = arr[off + got - 1] if got else 0
                ids = list(ids) + [ids[-1] if ids else -1] * (n - got)
                ts = list(ts) + [ts[-1] if ts else 0.0] * (n - got)
            b.ids += list(ids)
            b.ts += list(ts)
            b.streams += [src.stream] * n
            off += n
        self._filled[slot] = True
        return b

    def run(self) -> None:
        failures = 0
        while not self._stop.is_set():
            try:
                slot = self._free.get(timeout=0.1)
            except queue.Empty:
                continue
            try:
                b = self._fill(slot)
                failures = 0
            except StopIteration:
                self._ready.put(self._EOS)
                return
            except Exception as e:  # reference: a camera error killed the producer
                failures += 1
                if self.metrics is not None:
                    self.metrics.inc("source_errors")
                log.warning("feeder: source read failed (%d/%d): %s", failures, self.retry_limit, e)
                self._free.put(slot)
                if failures >= self.retry_limit:
                    self.error = e
                    self._ready.put(self._EOS)
                    return
                time.sleep(min(2.0, 0.05 * 2 ** failures))
                continue
            self.batches += 1
            self._ready.put(b)

    # --------------------------------------------------------------- consumer side
    def get(self, timeout: Optional[float] = None) -> Optional[Batch]:
        """Next filled batch; None at end of stream, feeder failure or stop() (and after
        ``timeout`` seconds, if given)."""
        try:
            b = self._ready.get(timeout=timeout)
        except queue.Empty:
            return None
        if b is self._EOS:
            self._ready.put(b)  # sticky: later calls see EOS too
            return None
        return b

    def release(self, b: Batch) -> None:
        self._free.put(b.slot)

    def stop(self) -> None:
        self._stop.set()
        self._ready.put(self._EOS)  # unblock a consumer waiting in get()
