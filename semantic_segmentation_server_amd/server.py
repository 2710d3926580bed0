"""Server entry point: ``python -m semantic_segmentation_server_amd.server [flags]``.

Reference bootstrap: ``serve()`` (``sem_seg_server.py:236-288``) — parse flags,
build the engine, load labels, probe the camera resolution, start the producer and
a gRPC server on ``[::]:50051`` sharing one 10-thread pool, then block on the
producer future.

Here the GPU pipeline runs in supervised worker processes, one per GPU (``--gpus N``;
``runtime/supervisor.py``), while this process -- which never touches the GPU -- hosts
the gRPC services and the result hub; ``--no_supervise`` runs it in-process (one GPU) or,
under torchrun, as one rank per GPU with the RCCL data path (``parallel/serving.py``).
The gRPC server has its own pool, both the v1 (reference-compatible) and v2 services are
registered, and metrics are dumped at exit when ``--metrics_dump`` is given.
"""
from __future__ import annotations

import logging
import os
import signal
import sys
import threading
import time
from typing import Optional

from . import config as C
from .api import service as S
from .labels import load_labels
from .runtime.engine import Engine
from .runtime.pipeline import Producer
from .runtime.results import ResultHub
from .runtime.sources import make_source, probe_resolution
from .utils.metrics import Metrics

log = logging.getLogger("semseg")


class Server:
    """In-process server (used by the CLI and by the integration tests)."""

    def __init__(self, cfg: C.Config, engine: Optional[Engine] = None, max_steps: Optional[int] = None):
        self.cfg = cfg
        self.metrics = Metrics()
        self.labels = load_labels(cfg.labels)
        self.hub = ResultHub(cfg.streams, cfg.buffer_max)
        self.camera_res = probe_resolution(cfg.source, cfg.camera_idx, cfg.camera_width,
                                           cfg.camera_height, cfg.source_path)
        self.engine = engine or Engine(cfg)
        from .utils.tracing import Tracer
        self.tracer = Tracer(self.metrics, enabled=cfg.profile)
        self.engine.tracer = self.tracer
        self.sources = [make_source(cfg.source, s, cfg.camera_idx, cfg.camera_width,
                                    cfg.camera_height, cfg.source_path, fps=cfg.fps_limit,
                                    seed=cfg.seed) for s in range(cfg.streams)]
        self.producer = Producer(self.engine, self.sources, self.hub, self.metrics, cfg.batch,
                                 max_steps=max_steps)
        self.grpc_server, self.port = S.make_server(cfg.max_workers, cfg.port, cfg.host)
        self.v1 = S.SemanticSegmentationServicer(self.hub, self.labels, cfg.num_detections,
                                                 self.camera_res, metrics=self.metrics)
        streams = [dict(stream_id=s.stream, width=s.resolution[0], height=s.resolution[1],
                        rank=0, source=cfg.source) for s in self.sources]
        self.v2 = S.SemanticSegmentationV2Servicer(self.hub, self.labels, cfg.num_detections,
                                                   streams, self.metrics, self._health)
        S.add_v1_servicer(self.v1, self.grpc_server)
        S.add_v2_servicer(self.v2, self.grpc_server)
        S.add_health_servicer(S.HealthServicer(lambda service: self._health()[0]), self.grpc_server)

    def _health(self):
        alive = self.producer.is_alive() and (time.time() - self.producer.alive_ts) < 30
        return alive, 1 if alive else 0, 1, "ok" if alive else f"producer down: {self.producer.error}"

    def start(self) -> "Server":
        self.grpc_server.start()
        self.producer.start()
        log.info("serving on port %d (%s backend, %s)", self.port, self.engine.backend,
                 self.engine.device)
        return self

    def stop(self, grace: Optional[float] = None) -> None:
        self.producer.stop()
        self.producer.join(timeout=30)
        self.grpc_server.stop(grace)
        for s in self.sources:
            s.close()
        if self.cfg.metrics_dump:
            self.metrics.dump(self.cfg.metrics_dump)

    def wait(self) -> None:
        # reference: block on the producer, then stop the server (:286-288)
        while self.producer.is_alive():
            self.producer.join(timeout=0.5)


def main(argv=None) -> int:
    cfg = C.apply_debug_env(C.parse(argv))
    logging.basicConfig(level=getattr(logging, cfg.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 or (cfg.gpus > 1 and not cfg.supervise):
        # torchrun launch (one process per GPU, rank 0 hosts gRPC): the RCCL data path
        # with P-1 group re-form (parallel/serving.py)
        from .parallel.serving import serve_distributed
        return serve_distributed(cfg)
    print("Loading {} with {} labels.".format(cfg.model or f"random-init {cfg.arch}", cfg.labels))
    if cfg.supervise and not cfg.debug_dump:
        # the GPU pipeline in supervised children (one per GPU, --gpus N): a faulted or
        # hung worker is replaced by a fresh process while the parent -- which never
        # touches the GPU -- keeps the gRPC services and the buffered results up
        from .runtime.supervisor import SupervisedServer
        sup = SupervisedServer(cfg).start()
        stop = threading.Event()
        signal.signal(signal.SIGTERM, lambda *a: stop.set())
        try:
            sup.wait(stop)
        except KeyboardInterrupt:
            pass
        sup.stop(None)
        return 0 if not sup.failed else 1
    srv = Server(cfg).start()
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *a: stop.set())
    try:
        while srv.producer.is_alive() and not stop.is_set():
            time.sleep(0.2)
    except KeyboardInterrupt:
        pass
    srv.stop(None)
    return 0


if __name__ == "__main__":
    sys.exit(main())
