"""Supervised worker (runtime/supervisor.py; VERDICT r3 Weak #10): a worker process that
dies mid-stream is replaced by a fresh child process, health goes back to SERVING and
records keep flowing into the parent's hub, which served the buffered records
throughout. CPU path (torch backend, synthetic camera): the supervision logic is the same
for a GPU worker, whose fault kills its process the same way."""
import time

import grpc
import pytest

from semantic_segmentation_server_amd import config as C
from semantic_segmentation_server_amd.api import proto as P
from semantic_segmentation_server_amd.runtime.supervisor import SupervisedServer


def _health(port):
    ch = grpc.insecure_channel(f"127.0.0.1:{port}")
    call = ch.unary_unary("/grpc.health.v1.Health/Check",
                          request_serializer=P.HealthCheckRequest.SerializeToString,
                          response_deserializer=P.HealthCheckResponse.FromString)
    r = call(P.HealthCheckRequest(service=""), timeout=5)
    ch.close()
    return r.status == P.HealthCheckResponse.SERVING


def test_worker_crash_is_replaced_by_a_fresh_process():
    cfg = C.Config(backend="torch", device="cpu", input_size=65, batch=1, port=0, host="127.0.0.1",
                   min_area_ratio=0.0005, inject_fault="worker:3", fps_limit=200.0, log_level="WARNING")
    sup = SupervisedServer(cfg, heartbeat_timeout_s=60.0).start()
    try:
        t_end = time.time() + 240
        while sup.metrics.counters.get("worker_restarts", 0) < 1 and time.time() < t_end:
            time.sleep(0.1)
        assert sup.metrics.counters.get("worker_restarts", 0) == 1, sup.error
        while not (sup.incarnation == 1 and sup.worker_up) and time.time() < t_end:
            time.sleep(0.1)
        pushed0 = sup.hub.buffers[0].pushed if 0 in sup.hub.buffers else 0
        steps0 = sup.worker_steps
        while (sup.worker_steps < steps0 + 3) and time.time() < t_end:
            time.sleep(0.1)
        assert sup.worker_up and sup.worker_steps >= steps0 + 3
        assert _health(sup.port)
        assert sup.alive and not sup.failed
        # the parent's hub kept what the first worker delivered and receives the second's
        assert sum(b.pushed for b in sup.hub.buffers.values()) >= pushed0
    finally:
        sup.stop(0)
    assert sup.finished  # a requested stop ends the worker cleanly (exit 0)
