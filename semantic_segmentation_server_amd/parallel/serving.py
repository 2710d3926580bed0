"""Multi-GPU serving: one process per GPU, rank 0 hosts the gRPC services.

Launch: ``torchrun --nproc-per-node N --master-addr 127.0.0.1 -m
semantic_segmentation_server_amd.server --gpus N [flags]``.

Every rank owns ``--streams`` frame sources (global stream id = rank * S + s) and
one engine on its GPU; each step a rank batches ``--batch`` frames from its
sources, runs the hipGraph-captured step, and the packed records plus frame
metadata are RCCL-gathered to rank 0, which pushes them into the per-stream
result hub behind the v1/v2 services. With ``--ingest scatter`` rank 0 owns the
sources for the whole node and RCCL-scatters frames instead.

Failure handling: every step starts with a tiny all-reduce that
carries the stop flag; a rank whose source fails keeps stepping on its last good
batch (logged) so collectives never hang. When a peer rank is lost, the next
collective fails (peer connection closed, or the ``--rank_timeout`` process-group
timeout) and rank 0 switches to degraded mode: it drops the process group,
re-shards onto itself (its own streams, local ingest) and keeps producing and
serving; Health/grpc.health report ``ranks_alive = 1`` and the cause
(``--no_degrade`` exits instead). A non-root rank that loses rank 0 exits.
``--inject_fault rank:step`` raises on that rank/step (used by tests).
"""
from __future__ import annotations

import logging
import signal
import threading
import time
from typing import List, Optional

import numpy as np
import torch

from . import dist as D
from .dp import DataParallelPipeline
from ..api import service as S
from ..config import Config
from ..labels import load_labels
from ..runtime.engine import Engine
from ..runtime.results import ResultHub
from ..runtime.sources import make_source
from ..utils.metrics import Metrics

log = logging.getLogger(__name__)


class DistributedServer:
    def __init__(self, cfg: Config, ctx: Optional[D.DistContext] = None,
                 max_steps: Optional[int] = None):
        self.cfg = cfg
        # RCCL only for the rank-0 frame scatter; otherwise a gloo group (records are
        # gathered from pinned host memory, and an initialised RCCL communicator alone
        # cost 23% of single-GPU throughput on MI355X -- see bench.py --pg)
        pg = "nccl" if cfg.ingest == "scatter" else "gloo"
        import torch
        self.ctx = ctx or D.init(pg, timeout_s=cfg.rank_timeout,
                                 device="cuda" if torch.cuda.is_available() and cfg.device != "cpu"
                                 else "auto")
        self.run_ctx = self.ctx  # == ctx until degraded to rank 0 alone
        self.degraded = False
        self.max_steps = max_steps
        self.metrics = Metrics()
        S_ = max(1, cfg.streams)
        self.S = S_
        own = cfg.ingest == "local" or self.ctx.is_root
        self.sources = [make_source(cfg.source, self.ctx.rank * S_ + s, cfg.camera_idx,
                                    cfg.camera_width, cfg.camera_height, cfg.source_path,
                                    fps=cfg.fps_limit, seed=cfg.seed) for s in range(S_)] if own else []
        res = (cfg.camera_width, cfg.camera_height) if not self.sources else self.sources[0].resolution
        self.camera_res = res
        self.engine = Engine(cfg, self.ctx.device)
        self.hub = ResultHub(self.ctx.world * S_, cfg.buffer_max) if self.ctx.is_root else None
        self.pipe = DataParallelPipeline(self.ctx, self.engine, res[0], res[1], cfg.batch,
                                         cfg.ingest, self.hub, S_)
        self.steps = 0
        self.alive = True
        self.error: Optional[str] = None
        self.grpc_server = None
        self.port = None
        self._last = None
        self._ingest = cfg.ingest
        self.fault = None
        if cfg.inject_fault:
            r, st = cfg.inject_fault.split(":")
            self.fault = (int(r), int(st))

    # ------------------------------------------------------------------ rpc
    def start_rpc(self) -> None:
        if not self.ctx.is_root:
            return
        labels = load_labels(self.cfg.labels)
        self.grpc_server, self.port = S.make_server(self.cfg.max_workers, self.cfg.port, self.cfg.host)
        S.add_v1_servicer(S.SemanticSegmentationServicer(self.hub, labels, self.cfg.num_detections,
                                                         self.camera_res, metrics=self.metrics),
                          self.grpc_server)
        streams = [dict(stream_id=r * self.S + s, width=self.camera_res[0],
                        height=self.camera_res[1], rank=r, source=self.cfg.source)
                   for r in range(self.ctx.world) for s in range(self.S)]
        S.add_v2_servicer(S.SemanticSegmentationV2Servicer(
            self.hub, labels, self.cfg.num_detections, streams, self.metrics,
            self._health), self.grpc_server)
        S.add_health_servicer(S.HealthServicer(lambda service: self.alive), self.grpc_server)
        self.grpc_server.start()
        log.info("rank 0 serving gRPC on port %d for %d ranks", self.port, self.ctx.world)

    def _health(self):
        alive = self.run_ctx.world if self.alive else 0
        return self.alive, alive, self.ctx.world, self.error or "ok"

    # ------------------------------------------------------------- degrade
    def _degrade(self, err: BaseException) -> None:
        """Peer lost: continue on rank 0 alone (local ingest, no collectives)."""
        log.error("rank 0 lost a peer (%r): degrading to single-rank serving", err)
        self.degraded = True
        self.error = f"degraded to rank 0 alone after: {err!r}"
        self.metrics.inc("degrade_events")
        try:
            D.destroy(self.ctx)
        except Exception:  # the group may already be broken
            pass
        self.run_ctx = D.DistContext(0, 1, self.ctx.local_rank, self.ctx.device, None)
        res = self.camera_res
        self.pipe = DataParallelPipeline(self.run_ctx, self.engine, res[0], res[1], self.cfg.batch,
                                         "local", self.hub, self.S)
        self._ingest = "local"

    # ----------------------------------------------------------------- step
    def _gather_local(self):
        if not self.sources:
            return None, None, None, None
        per = [self.cfg.batch // self.S + (1 if s < self.cfg.batch % self.S else 0)
               for s in range(self.S)]
        if self._ingest == "scatter":
            per = [p * self.run_ctx.world for p in per]
        imgs, ids, ts, strm = [], [], [], []
        for src, n in zip(self.sources, per):
            if n == 0:
                continue
            try:
                f, fid, t = src.read_batch(n)
            except StopIteration:
                raise
            except Exception as e:  # keep the collectives in lock-step: reuse the last batch
                log.warning("rank %d source %d failed: %s", self.ctx.rank, src.stream, e)
                self.metrics.inc("source_errors")
                if self._last is None:
                    raise
                return self._last
            imgs.append(f)
            ids += list(fid)
            ts += list(t)
            strm += [src.stream] * len(fid)
        out = (np.concatenate(imgs), ids, ts, strm)
        self._last = out
        return out

    def step(self) -> bool:
        """One lock-step iteration on every rank. Returns False when stopping."""
        if self.fault and self.fault == (self.ctx.rank, self.steps):
            raise RuntimeError(f"injected fault on rank {self.ctx.rank} at step {self.steps}")
        t0 = time.perf_counter()
        stop = 0.0
        try:
            frames, ids, ts, strm = self._gather_local()
        except StopIteration:
            stop, frames = 1.0, None
        if D.allreduce_max(self.run_ctx, stop) > 0:
            return False
        if frames is not None:
            host = torch.from_numpy(np.ascontiguousarray(frames))
            if self.engine.is_cuda:
                host = host.pin_memory()
            self.pipe.prefetch(host)
        local_ids = ids if self._ingest == "local" else None
        recs = self.pipe.step(local_ids, ts if local_ids else None, strm if local_ids else None)
        dt = (time.perf_counter() - t0) * 1e3
        n = self.cfg.batch * self.run_ctx.world
        self.metrics.inc("frames", n)
        self.metrics.inc("objects", len(recs))
        self.metrics.observe("step_ms", dt)
        self.metrics.observe("frame_ms", dt / n)
        self.steps += 1
        return self.max_steps is None or self.steps < self.max_steps

    def run(self, stop_event: Optional[threading.Event] = None) -> None:
        self.start_rpc()
        while True:
            try:
                while True:
                    if stop_event is not None and stop_event.is_set():
                        if D.allreduce_max(self.run_ctx, 1.0) > 0:
                            return
                    if not self.step():
                        return
            except Exception as e:
                injected_here = self.fault is not None and self.fault[0] == self.ctx.rank
                if (self.ctx.is_root and self.run_ctx.world > 1 and self.cfg.degrade
                        and not injected_here):
                    self._degrade(e)
                    continue  # keep stepping on rank 0 alone
                self.alive = False
                self.error = repr(e)
                log.exception("rank %d stopped", self.ctx.rank)
                raise

    def stop(self) -> None:
        if self.grpc_server is not None:
            self.grpc_server.stop(0)
        for s in self.sources:
            s.close()
        if self.cfg.metrics_dump and self.ctx.is_root:
            self.metrics.dump(self.cfg.metrics_dump)


def serve_distributed(cfg: Config) -> int:
    srv = DistributedServer(cfg)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *a: stop.set())
    try:
        srv.run(stop)
    except KeyboardInterrupt:
        pass
    finally:
        srv.stop()
        D.destroy(srv.ctx)
    return 0
