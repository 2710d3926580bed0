"""Supervised GPU workers: the serving process survives device-pipeline failures.

Reference: one process; when ``recognize_and_segment`` dies the future returns and the
whole server stops (``/root/reference/sem_seg_server.py:274-288``). A GPU fault usually
leaves the HIP context of the faulting process unusable, so recovering in-process is not
an option; SURVEY.md §5.3 asks that a per-GPU worker's death leave the service up.

The serving process is split in two:

  parent (never initialises the GPU)   gRPC v1 / v2 / health services, the result hub
                                       (``gpus * streams`` streams), metrics; supervises
                                       the workers
  worker r (one child per GPU)         its own sources (global stream ids r * S + s) ->
                                       engine on cuda:r -> the measured pipeline
                                       (``runtime/pipeline.py``: feeder, bound hipGraphs,
                                       split post-processing); records to the parent

Transport (one channel set per worker INCARNATION, never reused -- a worker that dies
inside a write cannot leave a lock held or half a message behind for its successor):

* records: a single-producer / single-consumer ring of ``RECORD_DTYPE`` rows in shared
  memory (``_RecordRing``; no pickling, one memcpy per step on each side); the worker
  publishes a chunk by advancing the write index after the rows, the parent advances
  the read index after copying them out. A full ring drops the chunk (counted).
* progress: the ring header carries the worker's step count and the time of its last
  step, written by the worker's producer loop itself -- liveness is step PROGRESS, not a
  timer thread, so a worker whose GPU hangs (producer stuck in a synchronize) goes stale
  and is replaced.
* control: a per-incarnation queue for the rare messages (up, metrics snapshot, error,
  done); a corrupt or truncated message restarts that worker instead of killing the
  monitor.

Restart policy: a worker that exits non-zero, goes stale (no step for
``heartbeat_timeout_s`` after its first step), or has not completed its first step
within ``startup_timeout_s`` (lazy plan build and autotune, hipGraph capture, priming
steps and the first camera frame all come before it) is
killed and replaced by a FRESH child process (never an exec of the faulted one), with
exponential backoff, at most ``max_restarts`` times per ``restart_window_s`` (per rank).
Health is SERVING while at least one rank is up (a rank that restarts or gave up costs
only its own streams: the others keep serving, and the detail says "degraded: up/total");
the v2 Health RPC reports ranks alive / total;
``worker_restarts`` counts the restarts. Records already in the hub keep being served
throughout. All workers exiting 0 (end of stream) ends the server, as in the reference.

Multi-GPU: the workers are independent data-parallel replicas -- each ingests its own
cameras and gathers nothing over a collective, so a lost rank costs only its own streams
while it restarts, and no survivor can be left blocked in a collective with a dead peer.
The unsupervised torchrun path (``parallel/serving.py``) keeps the RCCL frame scatter /
record gather and the P-1 group re-form.

Fault injection (tests): ``--inject_fault worker:N`` makes the first incarnation of every
worker exit abruptly (``os._exit``, like a crashed process) after N steps;
``worker:R:N`` only rank R's; ``hang:R:N`` makes rank R's producer stop stepping after N
steps while its process stays alive (a hung GPU); ``slowstart:R:S`` delays rank R's
first step by S seconds (a cold plan autotune or graph capture after "up").
"""
from __future__ import annotations

import logging
import multiprocessing as mp
import os
import queue as _queue
import threading
import time
from multiprocessing import shared_memory
from typing import List, Optional

import numpy as np

from ..config import Config
from .results import RECORD_DTYPE

log = logging.getLogger(__name__)


class _RecordRing:
    """SPSC ring of RECORD_DTYPE rows in POSIX shared memory.

    Header (int64 words): 0 write index (rows published), 1 read index (rows consumed),
    2 worker steps, 3 dropped rows, 4 last-step time (float64 bits, time.time()),
    5 capacity in rows.
    Indices only grow; slot = index % cap. The producer writes the rows, then the write
    index (x86-64 keeps stores in program order); the consumer reads the write index,
    copies the rows, then stores the read index."""

    HDR = 8

    def __init__(self, cap: int = 1 << 16, name: Optional[str] = None):
        self.cap = int(cap)
        nbytes = self.HDR * 8 + self.cap * RECORD_DTYPE.itemsize
        self.owner = name is None
        self.shm = shared_memory.SharedMemory(name=name, create=self.owner, size=nbytes if self.owner else 0)
        buf = self.shm.buf
        self.hdr = np.ndarray((self.HDR,), dtype=np.int64, buffer=buf)
        if self.owner:
            self.hdr[:] = 0
            self.hdr[5] = self.cap
        else:
            self.cap = int(self.hdr[5])  # the segment may be page-rounded: cap from the header
        self.rows = np.ndarray((self.cap,), dtype=RECORD_DTYPE, buffer=buf, offset=self.HDR * 8)
        self.ts = np.ndarray((1,), dtype=np.float64, buffer=buf, offset=4 * 8)
        if self.owner:
            self.ts[0] = time.time()

    @property
    def name(self) -> str:
        return self.shm.name

    # ---- worker side
    def push(self, recs: np.ndarray) -> bool:
        n = len(recs)
        if n == 0:
            return True
        w, r = int(self.hdr[0]), int(self.hdr[1])
        if n > self.cap - (w - r):
            self.hdr[3] += n
            return False
        s = w % self.cap
        k = min(n, self.cap - s)
        self.rows[s:s + k] = recs[:k]
        if k < n:
            self.rows[:n - k] = recs[k:]
        self.hdr[0] = w + n
        return True

    def progress(self, steps: int) -> None:
        self.hdr[2] = steps
        self.ts[0] = time.time()

    # ---- parent side
    def pull(self) -> np.ndarray:
        w, r = int(self.hdr[0]), int(self.hdr[1])
        n = w - r
        if n <= 0:
            return np.zeros(0, dtype=RECORD_DTYPE)
        s = r % self.cap
        k = min(n, self.cap - s)
        out = np.empty(n, dtype=RECORD_DTYPE)
        out[:k] = self.rows[s:s + k]
        if k < n:
            out[k:] = self.rows[:n - k]
        self.hdr[1] = w
        return out

    @property
    def steps(self) -> int:
        return int(self.hdr[2])

    @property
    def drops(self) -> int:
        return int(self.hdr[3])

    @property
    def last_step(self) -> float:
        return float(self.ts[0])

    def close(self) -> None:
        self.hdr = self.rows = self.ts = None
        try:
            self.shm.close()
        except Exception:  # pragma: no cover - views still exported
            pass
        if self.owner:
            try:
                self.shm.unlink()
            except FileNotFoundError:
                pass


class _RingHub:
    """The worker's stand-in for the ResultHub: pushes go to the shared-memory ring."""

    def __init__(self, ring: _RecordRing):
        self.ring = ring
        self.buffers = {}
        self.depth = 0

    def push_records(self, recs) -> None:
        if len(recs):
            self.ring.push(np.ascontiguousarray(recs))


def _fault_for(spec: Optional[str], rank: int, incarnation: int):
    """(kind, step) of the fault injected into this worker incarnation, or None."""
    if not spec or incarnation != 0:
        return None
    parts = spec.split(":")
    if parts[0] == "worker" and len(parts) == 2:
        return "crash", int(parts[1])
    if parts[0] in ("worker", "hang", "slowstart") and len(parts) == 3 and int(parts[1]) == rank:
        return {"worker": "crash"}.get(parts[0], parts[0]), float(parts[2])
    return None


def _worker_main(cfg: Config, rank: int, ring_name: str, q, stop_evt, incarnation: int,
                 max_steps: Optional[int]) -> None:
    """Child process: rank ``rank``'s producer, reporting through the ring and ``q``."""
    logging.basicConfig(level=getattr(logging, cfg.log_level.upper(), logging.INFO),
                        format=f"%(asctime)s %(levelname)s worker{rank}: %(message)s")
    os.environ["LOCAL_RANK"] = str(rank)
    from ..parallel.affinity import pin_to_gpu_numa
    pin_to_gpu_numa(rank)  # before this process touches the GPU
    import torch
    from ..utils.metrics import Metrics
    from .engine import Engine
    from .pipeline import Producer
    from .sources import make_source
    ring = _RecordRing(name=ring_name)
    metrics = Metrics()
    device = None
    if cfg.device != "cpu" and torch.cuda.is_available() and torch.cuda.device_count() > rank:
        device = torch.device("cuda", rank)
    engine = Engine(cfg, device)
    S = max(1, cfg.streams)
    sources = [make_source(cfg.source, rank * S + s, cfg.camera_idx, cfg.camera_width, cfg.camera_height,
                           cfg.source_path, fps=cfg.fps_limit, seed=cfg.seed + rank)
               for s in range(S)]
    prod = Producer(engine, sources, _RingHub(ring), metrics, cfg.batch, max_steps=max_steps)
    fault = _fault_for(cfg.inject_fault, rank, incarnation)

    def on_step(n: int) -> None:  # step progress, published by the producer thread itself
        ring.progress(n)
        if fault is not None and fault[0] == "hang" and n >= fault[1]:
            # a hung GPU: the producer thread blocks (as in a synchronize that never
            # returns) while the process and its other threads live on
            while not stop_evt.is_set():
                time.sleep(0.05)

    prod.on_step = on_step
    q.put(("up", rank, incarnation, f"{engine.backend} {engine.device}"))
    if fault is not None and fault[0] == "slowstart":
        time.sleep(fault[1])  # a first step that takes long (cold autotune, graph capture)
    prod.start()
    last_snap = 0.0
    while prod.is_alive():
        if stop_evt.is_set():
            prod.stop()
        if fault is not None and fault[0] == "crash" and prod.steps >= fault[1]:
            os._exit(70)  # a crashed worker: no cleanup, no goodbye
        now = time.time()
        if now - last_snap > 0.5:
            q.put(("snap", rank, metrics.snapshot()))
            last_snap = now
        prod.join(timeout=0.02)
    ring.progress(prod.steps)
    for s in sources:
        s.close()
    q.put(("snap", rank, metrics.snapshot()))
    if prod.error is not None:
        q.put(("error", rank, repr(prod.error)))
        q.close()
        q.join_thread()
        os._exit(3)
    q.put(("done", rank, prod.steps))
    q.close()
    q.join_thread()


class _Worker:
    """Parent-side state of one rank's current incarnation."""

    def __init__(self, rank: int):
        self.rank = rank
        self.incarnation = -1
        self.proc = None
        self.ring: Optional[_RecordRing] = None
        self.q = None
        self.up = False
        self.started = 0.0
        self.steps = 0
        self.progress_seen = 0.0
        self.finished = False
        self.failed = False
        self.error: Optional[str] = None
        self.restarts: List[float] = []
        self.restart_at: Optional[float] = None
        self.first_step = False  # the current incarnation has completed a step
        self.snap: dict = {}
        self.base: dict = {}  # counters of the retired incarnations (added to snap's)


class SupervisedServer:
    def __init__(self, cfg: Config, max_steps: Optional[int] = None, max_restarts: int = 5,
                 restart_window_s: float = 600.0, heartbeat_timeout_s: float = 120.0,
                 startup_timeout_s: float = 600.0, ring_rows: int = 1 << 16):
        from ..api import service as S
        from ..labels import load_labels
        from ..utils.metrics import Metrics
        from .results import ResultHub
        from .sources import probe_resolution
        self.cfg = cfg
        self.max_steps = max_steps
        self.max_restarts = max_restarts
        self.restart_window_s = restart_window_s
        self.heartbeat_timeout_s = heartbeat_timeout_s
        self.startup_timeout_s = startup_timeout_s
        self.ring_rows = ring_rows
        self.nw = max(1, int(cfg.gpus))
        self.S = max(1, cfg.streams)
        self.metrics = Metrics()
        self.hub = ResultHub(self.nw * self.S, cfg.buffer_max)
        self.camera_res = probe_resolution(cfg.source, cfg.camera_idx, cfg.camera_width,
                                           cfg.camera_height, cfg.source_path)
        self.grpc_server, self.port = S.make_server(cfg.max_workers, cfg.port, cfg.host)
        labels = load_labels(cfg.labels)
        S.add_v1_servicer(S.SemanticSegmentationServicer(self.hub, labels, cfg.num_detections,
                                                         self.camera_res, metrics=self.metrics),
                          self.grpc_server)
        streams = [dict(stream_id=r * self.S + s, width=self.camera_res[0], height=self.camera_res[1],
                        rank=r, source=cfg.source) for r in range(self.nw) for s in range(self.S)]
        S.add_v2_servicer(S.SemanticSegmentationV2Servicer(self.hub, labels, cfg.num_detections,
                                                           streams, self.metrics, self._health),
                          self.grpc_server)
        S.add_health_servicer(S.HealthServicer(lambda service: self._health()[0]), self.grpc_server)
        self._ctx = mp.get_context("spawn")
        self._stop = self._ctx.Event()
        self.workers = [_Worker(r) for r in range(self.nw)]
        self._mon = threading.Thread(target=self._monitor, name="supervisor", daemon=True)
        self._shutdown = threading.Event()

    # ------------------------------------------------------------ compat (1 GPU)
    @property
    def incarnation(self) -> int:
        return self.workers[0].incarnation

    @property
    def worker_up(self) -> bool:
        return self.workers[0].up

    @property
    def worker_steps(self) -> int:
        return self.workers[0].steps

    @property
    def error(self) -> Optional[str]:
        errs = [w.error for w in self.workers if w.error]
        return "; ".join(errs) if errs else None

    @property
    def finished(self) -> bool:
        return all(w.finished for w in self.workers)

    @property
    def failed(self) -> bool:
        return any(w.failed for w in self.workers) and not any(w.up for w in self.workers)

    # ------------------------------------------------------------------ workers
    def _spawn(self, w: _Worker) -> None:
        w.incarnation += 1
        w.up = False
        w.q = self._ctx.Queue()
        w.ring = _RecordRing(self.ring_rows)
        w.proc = self._ctx.Process(target=_worker_main, name=f"semseg-worker{w.rank}-{w.incarnation}",
                                   args=(self.cfg, w.rank, w.ring.name, w.q, self._stop, w.incarnation,
                                         self.max_steps), daemon=True)
        w.proc.start()
        w.started = time.time()
        w.progress_seen = w.started
        w.first_step = False
        w.restart_at = None
        log.info("worker %d incarnation %d started (pid %d)", w.rank, w.incarnation, w.proc.pid)

    def _health(self):
        """SERVING while any rank is up: a lost rank degrades the server (its streams
        pause) but the others keep serving."""
        up = sum(1 for w in self.workers if w.up and not self._stale(w))
        ok = up > 0
        if up == self.nw:
            detail = "ok"
        else:
            detail = f"degraded: {up}/{self.nw} workers up" + (f"; {self.error}" if self.error else "")
        return ok, up, self.nw, detail

    def _stale(self, w: _Worker) -> bool:
        """No step for heartbeat_timeout_s -- counted only after the incarnation's first
        step; until then the startup deadline applies."""
        return w.up and w.first_step and time.time() - w.progress_seen > self.heartbeat_timeout_s

    def _pull(self, w: _Worker) -> None:
        if w.ring is None:
            return
        recs = w.ring.pull()
        if len(recs):
            self.hub.push_records(recs)
            self.metrics.inc("objects", len(recs))
        st = w.ring.steps
        if st != w.steps:
            w.steps = st
            w.progress_seen = time.time()
        if st > 0 and not w.first_step:
            w.first_step = True
            w.progress_seen = time.time()

    def _drain(self, w: _Worker) -> None:
        """Control messages of the current incarnation. A message that fails to arrive
        whole (the worker died mid-write) marks that worker for a restart; the monitor
        thread itself never dies on it."""
        if w.q is None:
            return
        for _ in range(64):
            try:
                msg = w.q.get_nowait()
            except _queue.Empty:
                return
            except Exception as e:  # truncated / corrupt message from a dying worker
                w.error = f"worker {w.rank}: control channel broken ({e!r})"
                if w.proc is not None and w.proc.is_alive():
                    w.proc.kill()
                return
            kind = msg[0]
            if kind == "up":
                w.up = True
                w.progress_seen = time.time()
                log.info("worker %d incarnation %d up: %s", w.rank, msg[2], msg[3])
            elif kind == "snap":
                w.snap = msg[2]
                self._merge_snapshots()
            elif kind == "error":
                w.error = f"worker {w.rank}.{w.incarnation}: {msg[2]}"
            elif kind == "done":
                w.finished = True

    def _merge_snapshots(self) -> None:
        """Forward the workers' metrics into the parent's (--metrics_dump, v2 GetStats):
        counters summed over ranks as ``worker_<name>``; histogram summaries
        (frame_latency_ms, step_ms, buffer_depth, ...) as ``worker_<name>`` with one
        worker, ``worker<rank>_<name>`` with several."""
        ext: dict = {}
        for w in self.workers:
            for k, v in (w.snap or {}).items():
                if isinstance(v, dict):
                    ext[f"worker_{k}" if self.nw == 1 else f"worker{w.rank}_{k}"] = v
                elif isinstance(v, (int, float)) and k not in ("uptime_s", "fps"):
                    ext[f"worker_{k}"] = ext.get(f"worker_{k}", 0.0) + float(v)
            # retired incarnations' counters: totals never go backwards across a restart
            for k, v in w.base.items():
                ext[f"worker_{k}"] = ext.get(f"worker_{k}", 0.0) + v
        with self.metrics._lock:
            self.metrics.external = ext

    def _retire(self, w: _Worker) -> None:
        """After the process ended: deliver what it published, free its channels."""
        if w.proc is not None:
            w.proc.join(timeout=10)
        self._pull(w)
        self._drain(w)
        for k, v in (w.snap or {}).items():  # fold the incarnation's counters into the base
            if isinstance(v, (int, float)) and not isinstance(v, bool) and k not in ("uptime_s", "fps"):
                w.base[k] = w.base.get(k, 0.0) + float(v)
        # the histogram summaries stay until the next incarnation sends its own
        w.snap = {k: v for k, v in (w.snap or {}).items() if isinstance(v, dict)}
        self._merge_snapshots()
        if w.ring is not None:
            dropped = w.ring.drops
            if dropped:
                self.metrics.inc("ipc_drops", dropped)
            w.ring.close()
            w.ring = None
        if w.q is not None:
            try:
                w.q.close()
                w.q.cancel_join_thread()
            except Exception:
                pass
            w.q = None
        w.up = False

    def _check(self, w: _Worker) -> None:
        if w.finished and w.proc is None:
            return
        if w.proc is None:  # waiting out a restart backoff
            if w.restart_at is not None and time.time() >= w.restart_at and not self._stop.is_set():
                w.error = None
                self._spawn(w)
            return
        self._drain(w)
        self._pull(w)
        p = w.proc
        now = time.time()
        stale = self._stale(w)
        no_start = not (w.up and w.first_step) and now - w.started > self.startup_timeout_s
        if p.is_alive() and not stale and not no_start:
            return
        if p.is_alive():
            why = "stopped making progress" if stale else "did not complete a first step"
            log.error("worker %d incarnation %d %s; killing it", w.rank, w.incarnation, why)
            w.error = f"worker {w.rank}.{w.incarnation} {why}"
            p.kill()
        self._retire(w)
        code = p.exitcode
        w.proc = None
        if code == 0 and not stale and not no_start or w.finished or self._stop.is_set():
            log.info("worker %d finished (exit %s)", w.rank, code)
            w.finished = True
            return
        w.error = w.error or f"worker {w.rank}.{w.incarnation} exited with code {code}"
        log.error("%s", w.error)
        w.restarts = [t for t in w.restarts if now - t < self.restart_window_s]
        if len(w.restarts) >= self.max_restarts:
            log.error("worker %d restarted %d times in %.0f s: giving up", w.rank, len(w.restarts),
                      self.restart_window_s)
            w.failed = True
            w.finished = True
            return
        w.restart_at = now + min(10.0, 0.5 * 2 ** len(w.restarts))
        w.restarts.append(now)
        self.metrics.inc("worker_restarts")

    def _monitor(self) -> None:
        while not self._shutdown.is_set():
            busy = False
            for w in self.workers:
                try:
                    self._check(w)
                except Exception:  # the supervisor must outlive any one worker's failure
                    log.exception("supervising worker %d", w.rank)
                busy = busy or (w.ring is not None and int(w.ring.hdr[0]) != int(w.ring.hdr[1]))
            if all(w.finished for w in self.workers):
                return
            if not busy:
                self._shutdown.wait(0.002)

    # ------------------------------------------------------------------ control
    def start(self) -> "SupervisedServer":
        self.grpc_server.start()
        for w in self.workers:
            self._spawn(w)
        self._mon.start()
        log.info("supervised server on port %d (%d worker%s)", self.port, self.nw, "s" if self.nw > 1 else "")
        return self

    @property
    def alive(self) -> bool:
        return not (self.finished or all(w.failed for w in self.workers))

    def wait(self, stop_event: Optional[threading.Event] = None) -> None:
        while self.alive and not (stop_event is not None and stop_event.is_set()):
            time.sleep(0.2)

    def stop(self, grace: Optional[float] = None) -> None:
        self._stop.set()
        deadline = time.time() + 30
        for w in self.workers:
            p = w.proc
            if p is not None:
                p.join(timeout=max(0.1, deadline - time.time()))
                if p.is_alive():
                    p.kill()
                    p.join(timeout=10)
        self._shutdown.set()
        if self._mon.is_alive():
            self._mon.join(timeout=10)
        for w in self.workers:
            if w.proc is not None or w.ring is not None:
                self._retire(w)
                w.proc = None
            w.finished = True
        self.grpc_server.stop(grace)
        if self.cfg.metrics_dump:
            self.metrics.dump(self.cfg.metrics_dump)
