"""Producer loop: frame sources -> engine -> result buffers.

Reference: ``recognize_and_segment`` (``sem_seg_server.py:135-213``) — one thread,
one camera, batch 1, host post-processing, and error handling that cannot work
(the ``cv2.error`` handler raises ``KeyError`` on its own format string, ``:206-207``;
``KeyboardInterrupt`` is never delivered to a worker thread, ``:208-209``). End of
stream ends the producer and thereby the whole server (``:286-288``).

Here a ``Producer`` thread batches frames from one or more streams per step
(round-robin, ``cfg.batch`` frames), runs the engine, and pushes records into the
per-stream buffers of a ``ResultHub``. Source errors are logged and retried with
exponential backoff instead of killing the server; end of stream stops the
producer (and the server if ``exit_on_eos``).

On a GPU the producer runs the measured pipeline (``runtime/driver.py``: feeder
thread with a pinned ring -> ``DataParallelPipeline`` with lag 1, bound per-slot
hipGraphs and split post-processing), the same loop ``bench.py`` times. The
synchronous ``Engine.step`` loop remains for CPU serving and ``--debug_dump``.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import List, Optional

import numpy as np

from ..utils.metrics import Metrics
from .results import ResultHub
from .sources import FrameSource

log = logging.getLogger(__name__)


class Producer(threading.Thread):
    def __init__(self, engine, sources: List[FrameSource], hub: ResultHub, metrics: Metrics,
                 batch: int = 1, max_steps: Optional[int] = None, retry_limit: int = 10):
        super().__init__(name="producer", daemon=True)
        self.engine = engine
        self.sources = sources
        self.hub = hub
        self.metrics = metrics
        self.batch = max(1, int(batch))
        self.max_steps = max_steps
        self.retry_limit = retry_limit
        self._stop_evt = threading.Event()
        self.error: Optional[BaseException] = None
        self.steps = 0
        self.alive_ts = time.time()
        self.on_step = None  # optional progress hook, called with the step count after each step

    def stop(self) -> None:
        self._stop_evt.set()
        f = getattr(self, "feeder", None)
        if f is not None:
            f.stop()

    def _gather(self):
        """Round-robin ``batch`` frames over the live sources."""
        per = [self.batch // len(self.sources)] * len(self.sources)
        for i in range(self.batch % len(self.sources)):
            per[i] += 1
        imgs, ids, ts, streams = [], [], [], []
        for src, n in zip(self.sources, per):
            if n == 0:
                continue
            f, fid, t = src.read_batch(n)
            imgs.append(f)
            ids += list(fid)
            ts += list(t)
            streams += [src.stream] * len(fid)
        return np.concatenate(imgs), ids, ts, streams

    def _use_driver(self) -> bool:
        e = self.engine
        return bool(getattr(e, "is_cuda", False) and getattr(e, "debug", None) is None
                    and e.cfg.graph and e.cfg.contour_mode == "fast")

    def _run_driver(self) -> None:
        from ..parallel.dist import DistContext
        from ..parallel.dp import DataParallelPipeline
        from .driver import PipelineDriver
        from .feeder import BatchFeeder
        tr = getattr(self.engine, "tracer", None)
        ctx = DistContext(0, 1, 0, self.engine.device, None)
        w, h = self.sources[0].resolution
        feeder = BatchFeeder(self.sources, self.batch, metrics=self.metrics)
        feeder.start()
        self.feeder = feeder
        try:
            pipe = DataParallelPipeline(ctx, self.engine, w, h, self.batch, "local", self.hub,
                                        len(self.sources), lag=1)
            if tr is not None:
                pipe.tracer = tr
            pipe.metrics = self.metrics  # capture -> record frame latency (frame_latency_ms)
            drv = PipelineDriver(pipe, feeder, tr, self.metrics)
            first = drv.next_batch()
            if first is None:
                return
            drv.start(first)
            while not self._stop_evt.is_set():
                if self.max_steps is not None and self.steps >= self.max_steps:
                    break
                nxt = drv.next_batch()
                drv.step(nxt)
                self.steps += 1
                self.alive_ts = time.time()
                if self.on_step is not None:
                    self.on_step(self.steps)
                if nxt is None:
                    log.info("end of stream after %d steps", self.steps)
                    break
            drv.finish()
        except Exception as e:
            self.error = e
            self.metrics.inc("producer_errors")
            log.exception("device pipeline failed")
        finally:
            feeder.stop()

    def run(self) -> None:
        failures = 0
        self.hub_clear()
        if self._use_driver():
            self._run_driver()
            return
        while not self._stop_evt.is_set():
            if self.max_steps is not None and self.steps >= self.max_steps:
                break
            try:
                t0 = time.perf_counter()
                tr = getattr(self.engine, "tracer", None)
                if tr is None:
                    from ..utils.tracing import NULL_TRACER as tr
                with tr.stage("capture"):
                    frames, ids, ts, streams = self._gather()
                recs = self.engine.step(frames, ids, ts, streams)
                with tr.stage("publish"):
                    self.hub.push_records(recs)
                self.metrics.observe("objects_per_frame", len(recs) / max(1, len(ids)))
                self.metrics.observe("buffer_depth", self.hub.depth)
                dt = (time.perf_counter() - t0) * 1e3
                self.metrics.observe("frame_ms", dt / len(ids))
                self.metrics.observe("step_ms", dt)
                self.metrics.inc("frames", len(ids))
                self.metrics.inc("objects", len(recs))
                self.steps += 1
                self.alive_ts = time.time()
                if self.on_step is not None:
                    self.on_step(self.steps)
                failures = 0
            except StopIteration:
                log.info("end of stream after %d steps", self.steps)
                break
            except Exception as e:  # keep serving; back off and retry
                failures += 1
                self.metrics.inc("producer_errors")
                log.exception("producer step failed (%d/%d)", failures, self.retry_limit)
                if failures >= self.retry_limit:
                    self.error = e
                    break
                time.sleep(min(2.0, 0.05 * 2 ** failures))

    def hub_clear(self) -> None:
        # the reference clears its deque when the producer starts (sem_seg_server.py:137)
        for b in self.hub.buffers.values():
            b.clear()
