"""Supervised workers (runtime/supervisor.py; VERDICT r3 Weak #10, r4 #9): a
worker process that dies or hangs mid-stream is replaced by a fresh child process, health
goes back to SERVING and records keep flowing into the parent's hub, which served the
buffered records throughout; with several workers (one per GPU) only the lost rank's
streams pause. CPU path (torch backend, synthetic camera): the supervision logic is the
same for a GPU worker, whose fault kills its process the same way."""
import time

import grpc
import numpy as np
import pytest

from semantic_segmentation_server_amd import config as C
from semantic_segmentation_server_amd.api import proto as P
from semantic_segmentation_server_amd.runtime.results import RECORD_DTYPE
from semantic_segmentation_server_amd.runtime.supervisor import SupervisedServer, _RecordRing


def _health(port):
    ch = grpc.insecure_channel(f"127.0.0.1:{port}")
    call = ch.unary_unary("/grpc.health.v1.Health/Check",
                          request_serializer=P.HealthCheckRequest.SerializeToString,
                          response_deserializer=P.HealthCheckResponse.FromString)
    r = call(P.HealthCheckRequest(service=""), timeout=5)
    ch.close()
    return r.status == P.HealthCheckResponse.SERVING


def _cfg(**kw):
    base = dict(backend="torch", device="cpu", input_size=65, batch=1, port=0, host="127.0.0.1",
                min_area_ratio=0.0005, fps_limit=200.0, log_level="WARNING")
    base.update(kw)
    return C.Config(**base)


def _wait(cond, t_end):
    while not cond() and time.time() < t_end:
        time.sleep(0.05)
    return cond()


def test_record_ring_wraps_and_drops_when_full():
    ring = _RecordRing(cap=8)
    try:
        peer = _RecordRing(name=ring.name)  # the worker's attachment
        a = np.zeros(5, dtype=RECORD_DTYPE)
        a["frame"] = np.arange(5)
        assert peer.push(a)
        assert list(ring.pull()["frame"]) == [0, 1, 2, 3, 4]
        b = np.zeros(6, dtype=RECORD_DTYPE)
        b["frame"] = np.arange(10, 16)
        assert peer.push(b)                       # wraps around the end of the ring
        assert not peer.push(b[:3])               # 6 + 3 > 8: dropped, counted
        assert ring.drops == 3
        assert list(ring.pull()["frame"]) == list(range(10, 16))
        assert len(ring.pull()) == 0
        peer.progress(7)
        assert ring.steps == 7 and ring.last_step > 0
        peer.shm.close()
    finally:
        ring.close()


def test_worker_crash_is_replaced_by_a_fresh_process():
    sup = SupervisedServer(_cfg(inject_fault="worker:3"), heartbeat_timeout_s=60.0).start()
    try:
        t_end = time.time() + 240
        assert _wait(lambda: sup.metrics.counters.get("worker_restarts", 0) >= 1, t_end), sup.error
        assert sup.metrics.counters.get("worker_restarts", 0) == 1
        assert _wait(lambda: sup.incarnation == 1 and sup.worker_up, t_end)
        pushed0 = sum(b.pushed for b in sup.hub.buffers.values())
        steps0 = sup.worker_steps
        assert _wait(lambda: sup.worker_steps >= steps0 + 3, t_end)
        assert _wait(lambda: _health(sup.port), t_end)
        assert sup.alive and not sup.failed
        # the parent's hub kept what the first worker delivered and receives the second's
        assert _wait(lambda: sum(b.pushed for b in sup.hub.buffers.values()) > pushed0, t_end)
        # the worker's own metrics (histograms included) reach the parent's registry
        assert _wait(lambda: sup.metrics.snapshot().get("worker_frames", 0) > 0, t_end)
        snap = sup.metrics.snapshot()
        assert "worker_step_ms" in snap, sorted(snap)
    finally:
        sup.stop(0)
    assert sup.finished  # a requested stop ends the worker cleanly (exit 0)


def test_rank0_worker_lost_at_world3_records_and_health_recover():
    """Three workers (one per GPU in production); rank 0's worker crashes. The other two
    keep delivering their streams throughout, rank 0 comes back as a fresh process and its
    stream resumes; health goes NOT_SERVING -> SERVING; the gRPC front-end never stops."""
    sup = SupervisedServer(_cfg(gpus=3, inject_fault="worker:0:4"), heartbeat_timeout_s=60.0).start()
    try:
        t_end = time.time() + 300
        assert _wait(lambda: all(w.up for w in sup.workers), t_end)
        assert _wait(lambda: sup.metrics.counters.get("worker_restarts", 0) >= 1, t_end), sup.error
        w0 = sup.workers[0]
        # the survivors' streams (global ids 1, 2) keep growing while rank 0 restarts
        others = lambda: sum(sup.hub.buffers[s].pushed for s in (1, 2) if s in sup.hub.buffers)
        o0 = others()
        assert _wait(lambda: others() > o0, t_end)
        assert _wait(lambda: w0.incarnation == 1 and w0.up, t_end)
        p0 = sup.hub.buffers[0].pushed if 0 in sup.hub.buffers else 0
        assert _wait(lambda: 0 in sup.hub.buffers and sup.hub.buffers[0].pushed > p0, t_end)
        assert _wait(lambda: _health(sup.port), t_end)
        ok, up, total, _ = sup._health()
        assert ok and (up, total) == (3, 3)
        assert [w.incarnation for w in sup.workers] == [1, 0, 0]
    finally:
        sup.stop(0)


def test_hung_worker_is_detected_by_progress_and_replaced():
    """A worker whose producer stops stepping (a hung GPU: the process stays alive and its
    threads keep running) is stale after heartbeat_timeout_s of no progress and is
    killed and replaced (liveness tied to step progress)."""
    sup = SupervisedServer(_cfg(gpus=2, inject_fault="hang:1:3"), heartbeat_timeout_s=3.0).start()
    try:
        t_end = time.time() + 240
        w1 = sup.workers[1]
        assert _wait(lambda: w1.incarnation == 1, t_end), sup.error
        assert "progress" in (w1.error or "") or sup.metrics.counters.get("worker_restarts", 0) >= 1
        assert _wait(lambda: w1.up and w1.steps >= 2, t_end)
        assert _wait(lambda: _health(sup.port), t_end)
        assert sup.workers[0].incarnation == 0
    finally:
        sup.stop(0)


def test_slow_first_step_is_not_stale():
    """the progress deadline starts at the incarnation's first step. A first
    step that takes longer than heartbeat_timeout_s (cold autotune, graph capture) is
    under the startup deadline, so the worker is not killed."""
    sup = SupervisedServer(_cfg(inject_fault="slowstart:0:4"), heartbeat_timeout_s=1.5,
                           startup_timeout_s=120.0).start()
    try:
        t_end = time.time() + 240
        assert _wait(lambda: sup.worker_steps >= 3, t_end), sup.error
        assert sup.incarnation == 0 and sup.metrics.counters.get("worker_restarts", 0) == 0
    finally:
        sup.stop(0)


def test_counters_survive_a_restart_and_health_degrades():
    """Retired incarnations' counters stay in the totals (they never go backwards), and a
    rank that is down leaves the server SERVING but degraded while another rank is up."""
    from semantic_segmentation_server_amd.runtime.supervisor import _Worker
    from semantic_segmentation_server_amd.utils.metrics import Metrics
    sup = SupervisedServer.__new__(SupervisedServer)
    sup.nw, sup.metrics, sup.heartbeat_timeout_s = 2, Metrics(), 60.0
    sup.workers = [_Worker(0), _Worker(1)]
    for w in sup.workers:
        w.up, w.first_step, w.progress_seen = True, True, time.time()
    sup.workers[0].snap = {"frames": 100.0, "step_ms": {"p50": 1.0}}
    sup.workers[1].snap = {"frames": 50.0}
    sup._merge_snapshots()
    assert sup.metrics.snapshot()["worker_frames"] == 150.0
    w0 = sup.workers[0]
    sup._retire(w0)                      # incarnation 0 ends after 100 frames
    w0.snap = {"frames": 7.0}            # the fresh incarnation starts from zero
    sup._merge_snapshots()
    assert sup.metrics.snapshot()["worker_frames"] == 157.0
    ok, up, total, detail = sup._health()
    assert ok and (up, total) == (1, 2) and detail.startswith("degraded: 1/2")
    sup.workers[1].up = False
    assert not sup._health()[0]
