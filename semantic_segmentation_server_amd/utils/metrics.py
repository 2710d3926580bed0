"""Counters and latency histograms.

The reference has no metrics at all (``print`` only, ``sem_seg_server.py:262,207``).
Here every pipeline stage reports into a ``Metrics`` registry that backs the v2
``GetStats`` RPC, the bench JSON and the at-exit dump.
"""
from __future__ import annotations

import json
import threading
import time
from collections import defaultdict
from typing import Dict, List

import numpy as np


class Reservoir:
    """Fixed-size ring of recent samples; percentiles over the window."""

    def __init__(self, size: int = 8192):
        self.buf = np.zeros(size, dtype=np.float64)
        self.n = 0

    def add(self, v: float) -> None:
        self.buf[self.n % len(self.buf)] = v
        self.n += 1

    def add_many(self, vs) -> None:
        """add() of every value of ``vs``, in order (one numpy scatter, not a Python loop;
        a few values: plain add()s, cheaper than the scatter's call overhead)."""
        if isinstance(vs, list) and len(vs) <= 8:
            L = len(self.buf)
            for v in vs:
                self.buf[self.n % L] = v
                self.n += 1
            return
        vs = np.asarray(vs, dtype=np.float64).ravel()
        L = len(self.buf)
        if len(vs) > L:  # only the last L can survive
            self.n += len(vs) - L
            vs = vs[-L:]
        self.buf[(self.n + np.arange(len(vs))) % L] = vs
        self.n += len(vs)

    def values(self) -> np.ndarray:
        return self.buf[: min(self.n, len(self.buf))]

    def summary(self) -> Dict[str, float]:
        v = self.values()
        if len(v) == 0:
            return {"count": 0}
        return {"count": int(self.n), "mean": float(v.mean()), "p50": float(np.percentile(v, 50)),
                "p90": float(np.percentile(v, 90)), "p99": float(np.percentile(v, 99)),
                "max": float(v.max())}


class Metrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.counters: Dict[str, float] = defaultdict(float)
        self.hists: Dict[str, Reservoir] = {}
        self.external: Dict[str, object] = {}  # entries forwarded from worker processes
        self.t_start = time.time()

    def inc(self, name: str, v: float = 1.0) -> None:
        with self._lock:
            self.counters[name] += v

    def observe(self, name: str, v: float) -> None:
        with self._lock:
            h = self.hists.get(name)
            if h is None:
                h = self.hists[name] = Reservoir()
            h.add(v)

    def observe_many(self, name: str, vs) -> None:
        with self._lock:
            h = self.hists.get(name)
            if h is None:
                h = self.hists[name] = Reservoir()
            h.add_many(vs)

    def timer(self, name: str):
        return _Timer(self, name)

    def snapshot(self) -> Dict:
        with self._lock:
            elapsed = max(time.time() - self.t_start, 1e-9)
            snap: Dict = dict(self.counters)
            snap["uptime_s"] = elapsed
            snap["fps"] = self.counters.get("frames", 0.0) / elapsed
            for k, h in self.hists.items():
                snap[k] = h.summary()
            snap.update(self.external)
        return snap

    def dump(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.snapshot(), f, indent=1, default=float)


class _Timer:
    def __init__(self, m: Metrics, name: str):
        self.m, self.name = m, name

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.m.observe(self.name, (time.perf_counter() - self.t0) * 1e3)


def percentile_ms(samples: List[float], q: float) -> float:
    return float(np.percentile(np.asarray(samples), q)) if samples else float("nan")
