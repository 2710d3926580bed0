"""Pipeline-stage tracing.

The reference has no timers at all; the only timing source it had, the Edge TPU
latency returned by ``run_inference``, is discarded (``sem_seg_server.py:162``).

``Tracer.stage(name)`` brackets one pipeline stage (ingest / model / post / D2H /
record build / RPC) with
  * a roctx range (``torch.cuda.nvtx`` is backed by roctx on ROCm builds), so the
    stages show up as markers next to the kernels in a ``rocprofv3
    --marker-trace --kernel-trace`` timeline;
  * host wall time -> ``Metrics`` histogram ``stage.<name>.host_ms``;
  * optionally device time: HIP events recorded on the current stream around the
    stage, resolved lazily (``flush``) so tracing never forces a synchronisation
    -> ``stage.<name>.gpu_ms``.
Disabled (the default; ``--profile`` enables it) every call is a no-op.
"""
from __future__ import annotations

import contextlib
import time
from collections import deque
from typing import Deque, Optional, Tuple

import torch

try:  # roctx via torch's nvtx shim (ROCm builds route it to roctracer)
    from torch.cuda import nvtx as _nvtx
    _nvtx.range_push("probe")
    _nvtx.range_pop()
    _HAS_RANGES = True
except Exception:  # pragma: no cover - CPU-only / stripped builds
    _HAS_RANGES = False


class Tracer:
    def __init__(self, metrics=None, enabled: bool = False, gpu_events: bool = True):
        self.metrics = metrics
        self.enabled = bool(enabled)
        self.gpu_events = bool(gpu_events) and torch.cuda.is_available()
        self._pending: Deque[Tuple[str, "torch.cuda.Event", "torch.cuda.Event"]] = deque()

    @contextlib.contextmanager
    def stage(self, name: str, stream: Optional["torch.cuda.Stream"] = None):
        if not self.enabled:
            yield
            return
        if _HAS_RANGES:
            _nvtx.range_push(name)
        ev0 = ev1 = None
        if self.gpu_events:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record(stream) if stream is not None else ev0.record()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            dt = (time.perf_counter() - t0) * 1e3
            if self.gpu_events:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record(stream) if stream is not None else ev1.record()
                self._pending.append((name, ev0, ev1))
            if _HAS_RANGES:
                _nvtx.range_pop()
            if self.metrics is not None:
                self.metrics.observe(f"stage.{name}.host_ms", dt)
            self.flush()

    def flush(self, block: bool = False) -> None:
        """Move completed device timings into the metrics (non-blocking unless asked)."""
        while self._pending:
            name, e0, e1 = self._pending[0]
            if not block and not e1.query():
                break
            if block:
                e1.synchronize()
            self._pending.popleft()
            if self.metrics is not None:
                self.metrics.observe(f"stage.{name}.gpu_ms", e0.elapsed_time(e1))


NULL_TRACER = Tracer(enabled=False)
