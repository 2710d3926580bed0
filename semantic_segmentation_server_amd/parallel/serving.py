"""Multi-GPU serving: one process per GPU, rank 0 hosts the gRPC services.

Launch: ``torchrun --nproc-per-node N --master-addr 127.0.0.1 -m
semantic_segmentation_server_amd.server --gpus N [flags]``.

Every rank owns ``--streams`` frame sources (global stream id = launch rank * S + s) and
one engine on its GPU. Each rank's loop is the measured pipeline (``runtime/driver.py``):
a feeder thread fills a ring of pinned batches, ``DataParallelPipeline`` (lag 1, bound
per-slot hipGraphs, post-processing on its own stream) runs the step and gathers the
packed records plus frame metadata to rank 0 -- with P-1 degradation on (the default)
from pinned host memory over gloo (a latency-bound ~41 KB per rank and step that the
host thread's slack absorbs); with ``--no_degrade`` or ``--gather rccl`` as one RCCL
gather of a packed device row on the result stream -- which pushes them into the
per-stream result hub behind the v1/v2 services. With ``--ingest scatter`` rank 0 owns
the sources for the whole node and scatters frames over RCCL (xGMI) and their metadata
over gloo instead. The per-step heartbeat is a gloo all-reduce of a host flag. (The CLI
default for several GPUs is the supervised form, ``runtime/supervisor.py``.)

Failure handling: every step starts with a tiny all-reduce carrying the
stop flag; a source error is retried by the feeder (the rank keeps stepping). When a
peer is lost, the next collective fails (peer connection closed, or the
``--rank_timeout`` process-group timeout) on every survivor, and the survivors RE-FORM
the group (``dist.reform``: membership agreed through a store hosted by launch rank 0,
renumbered by launch rank, a fresh process group of the next generation). Each survivor
keeps its own streams (their global ids do not change), so a lost rank costs exactly its
own cameras; Health / grpc.health report ``ranks_alive`` of the new group. If launch rank
0 is lost the others exit (it hosts the RPC). ``--no_degrade`` exits instead of
re-forming. ``--inject_fault rank:step`` raises on that (launch) rank / step (tests).
"""
from __future__ import annotations

import logging
import os
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
from ..runtime.driver import PipelineDriver
from ..runtime.engine import Engine
from ..runtime.feeder import BatchFeeder
from ..runtime.results import ResultHub
from ..runtime.sources import make_source
from ..utils.metrics import Metrics
from ..utils.tracing import Tracer

log = logging.getLogger(__name__)


class DistributedServer:
    def __init__(self, cfg: Config, ctx: Optional[D.DistContext] = None,
                 max_steps: Optional[int] = None):
        self.cfg = cfg
        # multi-GPU data path over RCCL (record gather, frame scatter) with a gloo group
        # beside it for the heartbeat / control traffic; gloo alone on CPU ranks or when
        # the host gather is asked for
        gpu = torch.cuda.is_available() and cfg.device != "cpu"
        # record gather: with P-1 degradation on (the serving default) the gather stays on
        # the host (pinned memory over gloo). An RCCL gather kernel whose peer died never
        # completes, and the survivors' result streams would stay blocked behind it after
        # the group is re-formed; --no_degrade (or --gather rccl) keeps the
        # RCCL data path, which bench.py measures. The pipeline's completion wait polls
        # for a peer's abort key on that path, so a lost peer still surfaces as PeerLost.
        # auto: RCCL (xGMI) on GPUs at N > 1 with --no_degrade, else the host gather
        world = int(os.environ.get("WORLD_SIZE", "1"))
        self.gather = cfg.gather if cfg.gather != "auto" else (
            "rccl" if gpu and world > 1 and not cfg.degrade
            and os.environ.get("SSA_SHARE_GPU", "0") != "1" else "host")
        # SSA_SHARE_GPU=1 (several ranks on one GPU, a rehearsal): RCCL refuses that, gloo
        share = os.environ.get("SSA_SHARE_GPU", "0") == "1"
        if share and cfg.ingest == "scatter":
            log.warning("--ingest scatter needs RCCL, which SSA_SHARE_GPU=1 rules out: local ingest")
            cfg.ingest = "local"
        pg = "nccl" if gpu and not share and (cfg.ingest == "scatter" or self.gather == "rccl") else "gloo"
        self.ctx = ctx or D.init(pg, timeout_s=cfg.rank_timeout,
                                 device="cuda" if torch.cuda.is_available() and cfg.device != "cpu"
                                 else "auto")
        self.run_ctx = self.ctx  # the current group (re-formed after a rank loss)
        self.launch_world = self.ctx.world
        self.degraded = False
        self.max_steps = max_steps
        self.metrics = Metrics()
        self.tracer = Tracer(self.metrics, enabled=cfg.profile)
        S_ = max(1, cfg.streams)
        self.S = S_
        me = self.ctx.orig_rank
        own = cfg.ingest == "local" or self.ctx.is_root
        self.sources = [make_source(cfg.source, me * S_ + s, cfg.camera_idx,
                                    cfg.camera_width, cfg.camera_height, cfg.source_path,
                                    fps=cfg.fps_limit, seed=cfg.seed) for s in range(S_)] if own else []
        res = (cfg.camera_width, cfg.camera_height) if not self.sources else self.sources[0].resolution
        self.camera_res = res
        self.engine = Engine(cfg, self.ctx.device)
        self.engine.tracer = self.tracer
        self.hub = ResultHub(self.ctx.world * S_, cfg.buffer_max) if self.ctx.is_root else None
        self._ingest = cfg.ingest
        self.feeder: Optional[BatchFeeder] = None
        self.driver: Optional[PipelineDriver] = None
        self._build_pipeline()
        self.steps = 0
        self.alive = True
        self.error: Optional[str] = None
        self.grpc_server = None
        self.port = None
        self.fault = None
        if cfg.inject_fault:
            r, st = cfg.inject_fault.split(":")
            self.fault = (int(r), int(st))

    def _build_pipeline(self) -> None:
        ctx = self.run_ctx
        if self.feeder is not None:
            self.feeder.stop()
        nb = self.cfg.batch * (ctx.world if self._ingest == "scatter" else 1)
        self.feeder = BatchFeeder(self.sources, nb, metrics=self.metrics) if self.sources else None
        if self.feeder is not None:
            self.feeder.start()
        pipe = DataParallelPipeline(ctx, self.engine, self.camera_res[0], self.camera_res[1],
                                    self.cfg.batch, self._ingest, self.hub, self.S, lag=1,
                                    gather=self.gather)
        pipe.tracer = self.tracer
        pipe.metrics = self.metrics
        pipe.rank_timeout_s = float(self.cfg.rank_timeout)
        self.driver = PipelineDriver(pipe, self.feeder, self.tracer, self.metrics)
        self._started = False

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
        return self.alive, alive, self.launch_world, self.error or "ok"

    # ------------------------------------------------------------- failure
    def _reform(self, err: BaseException) -> None:
        """Peer lost: re-form the group from the survivors and keep serving."""
        log.error("launch rank %d: collective failed (%r); re-forming the group",
                  self.ctx.orig_rank, err)
        self.metrics.inc("degrade_events")
        t0 = time.perf_counter()
        if self.driver is not None:
            try:
                self.driver.pipe.close(abort=True)  # its RCCL communicators include the lost peer
            except Exception:
                log.exception("closing the old pipeline's communicators")
        new = D.reform(self.run_ctx, timeout_s=self.cfg.rank_timeout)
        log.info("re-formed the group in %.2f s", time.perf_counter() - t0)
        self.degraded = True
        self.error = (f"degraded to {new.world}/{self.launch_world} ranks "
                      f"(launch ranks {new.members}) after: {err!r}")
        log.error("group re-formed: %s", self.error)
        self.run_ctx = new
        self._build_pipeline()

    # ----------------------------------------------------------------- step
    def step(self) -> bool:
        """One lock-step iteration on every rank. Returns False when stopping."""
        if self.fault and self.fault == (self.ctx.orig_rank, self.steps):
            raise RuntimeError(f"injected fault on rank {self.ctx.orig_rank} at step {self.steps}")
        if not self._started:
            first = self.driver.next_batch()
            eos = 1.0 if (self.feeder is not None and first is None) else 0.0
            if D.allreduce_max(self.run_ctx, eos) > 0:
                return False
            self.driver.start(first)
            self._started = True
        nxt = self.driver.next_batch()
        stop = 1.0 if (self.feeder is not None and nxt is None) else 0.0
        if D.allreduce_max(self.run_ctx, stop) > 0:
            self.driver.step(None)     # the in-flight batch still runs (collected by finish)
            return False
        self.driver.step(nxt)
        self.steps += 1
        return self.max_steps is None or self.steps < self.max_steps

    def run(self, stop_event: Optional[threading.Event] = None) -> None:
        self.start_rpc()
        while True:
            try:
                while True:
                    if stop_event is not None and stop_event.is_set():
                        if D.allreduce_max(self.run_ctx, 1.0) > 0:
                            self.driver.finish()
                            return
                    if not self.step():
                        self.driver.finish()
                        return
            except Exception as e:
                injected_here = self.fault is not None and self.fault[0] == self.ctx.orig_rank
                if (self.run_ctx.world > 1 and self.cfg.degrade and not injected_here
                        and self.run_ctx.store is not None):
                    try:
                        self._reform(e)
                        continue  # keep stepping in the re-formed group
                    except Exception as e2:
                        log.error("re-forming failed: %r", e2)
                        e = e2
                self.alive = False
                self.error = repr(e)
                log.exception("rank %d stopped", self.ctx.orig_rank)
                raise

    def stop(self) -> None:
        if self.grpc_server is not None:
            self.grpc_server.stop(0)
        if self.feeder is not None:
            self.feeder.stop()
        for s in self.sources:
            s.close()
        if self.cfg.metrics_dump and self.ctx.is_root:
            self.metrics.dump(self.cfg.metrics_dump)


def serve_distributed(cfg: Config) -> int:
    from .affinity import pin_to_gpu_numa
    pin_to_gpu_numa()  # before the first GPU call of this process
    srv = DistributedServer(cfg)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *a: stop.set())
    try:
        srv.run(stop)
    except KeyboardInterrupt:
        pass
    finally:
        srv.stop()
        D.destroy(srv.run_ctx)
    return 0
