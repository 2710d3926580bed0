"""T6: data-parallel pipeline on a fake cluster (gloo, CPU, world sizes 2 and 3).

The per-rank engine is replaced by a deterministic fake that encodes which frames
it saw into its packed records, so the test checks the collective plumbing:
rank-0 scatter of the node batch (X1), record gather to rank 0 (X2), stream-id
assignment and push into the result hub, and max-over-ranks timing (X3).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


class FakeCfg:
    max_segments = 4


class FakeEngine:
    def __init__(self):
        self.cfg = FakeCfg()
        self.device = torch.device("cpu")

    def set_camera(self, w, h):
        self.cam = (w, h)

    def run_device(self, frames):
        B = frames.shape[0]
        K = self.cfg.max_segments
        packed = torch.zeros(B, 1 + 5 * K)
        for i in range(B):
            v = float(frames[i, 0, 0, 0])          # frame tag written by the test
            packed[i, 0] = 1
            packed[i, 1:6] = torch.tensor([15.0, 0.5, 0.1, v / 255.0, 0.25])
        return None, packed


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ingest, q, lag=0, gather="host"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from semantic_segmentation_server_amd.parallel import dist as D
    from semantic_segmentation_server_amd.parallel.dp import DataParallelPipeline
    from semantic_segmentation_server_amd.runtime.results import ResultHub
    ctx = D.init("gloo")
    B = 2
    hub = ResultHub(world) if ctx.is_root else None
    pipe = DataParallelPipeline(ctx, FakeEngine(), 8, 6, B, ingest, hub, lag=lag, gather=gather)
    if ingest == "scatter":
        nb = B * world if ctx.is_root else B
        frames = torch.zeros(nb, 6, 8, 3, dtype=torch.uint8)
        if ctx.is_root:
            for i in range(nb):
                frames[i, 0, 0, 0] = 10 + i
    else:
        frames = torch.zeros(B, 6, 8, 3, dtype=torch.uint8)
        for i in range(B):
            frames[i, 0, 0, 0] = 10 + rank * B + i
    pipe.prefetch(frames)
    recs = pipe.step()
    # default frame ids advance per step by the frames of one rank (local ingest) or of
    # the whole node (scatter: ids are rank 0's node-level capture ids)
    adv = B * world if ingest == "scatter" else B
    if lag:  # records arrive `lag` steps late; the later steps' come with flush()
        assert len(recs) == 0
        for k in range(lag):
            pipe.prefetch(frames)
            recs = pipe.step()
            assert len(recs) == 0 or k == lag - 1
        last = pipe.flush()
        if ctx.is_root:
            n = len(recs)
            assert n > 0 and len(last) == lag * n
            for j in range(lag):
                part = last[j * n:(j + 1) * n]
                assert np.array_equal(part["cx"], recs["cx"]) and np.all(part["frame"] == recs["frame"] + (j + 1) * adv)
    t = D.allreduce_max(ctx, float(rank))
    if ctx.is_root:
        q.put((recs["cx"].tolist(), recs["stream"].tolist(), t, hub.depth))
    D.barrier(ctx)
    D.destroy(ctx)


@pytest.mark.parametrize("world,ingest,lag,gather", [
    (2, "local", 0, "host"), (2, "scatter", 0, "host"), (3, "scatter", 0, "host"),
    (2, "local", 1, "host"), (2, "scatter", 1, "host"), (2, "local", 1, "rccl"),
    (3, "scatter", 0, "rccl"), (2, "local", 2, "host"), (2, "scatter", 2, "host")])
def test_dp_gather_and_scatter(world, ingest, lag, gather):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ingest, q, lag, gather))
             for r in range(world)]
    for p in procs:
        p.start()
    cx, streams, tmax, depth = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    B = 2
    exp = [(10 + i) / 255.0 for i in range(world * B)]
    assert np.allclose(cx, exp, atol=1e-6)          # frame i went to rank i // B, came back in order
    assert streams == [i // B for i in range(world * B)]
    assert tmax == world - 1
    assert depth == world * B * (lag + 1)


def _scatter_meta_worker(rank, world, port, q):
    """Scatter ingest with real capture metadata on rank 0: every record must carry the
    id / timestamp / source stream of the frame it came from."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from semantic_segmentation_server_amd.parallel import dist as D
    from semantic_segmentation_server_amd.parallel.dp import DataParallelPipeline
    from semantic_segmentation_server_amd.runtime.results import ResultHub
    ctx = D.init("gloo")
    B = 2
    hub = ResultHub(8) if ctx.is_root else None
    pipe = DataParallelPipeline(ctx, FakeEngine(), 8, 6, B, "scatter", hub, lag=1)
    nb = B * world if ctx.is_root else B
    frames = torch.zeros(nb, 6, 8, 3, dtype=torch.uint8)
    ids = ts = st = None
    if ctx.is_root:
        for i in range(nb):
            frames[i, 0, 0, 0] = 10 + i
        ids = [1000 + 7 * i for i in range(nb)]
        ts = [50.0 + i for i in range(nb)]
        st = [5 if i % 2 else 3 for i in range(nb)]   # two cameras on rank 0
    pipe.prefetch(frames)
    pipe.step(ids, ts, st)
    recs = pipe.flush()
    if ctx.is_root:
        q.put((recs["cx"].tolist(), recs["frame"].tolist(), recs["ts"].tolist(), recs["stream"].tolist()))
    D.barrier(ctx)
    D.destroy(ctx)


def test_scatter_keeps_capture_metadata():
    world, B = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_meta_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    cx, frame, ts, stream = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = world * B
    assert np.allclose(cx, [(10 + i) / 255.0 for i in range(n)], atol=1e-6)
    assert frame == [1000 + 7 * i for i in range(n)]
    assert ts == [50.0 + i for i in range(n)]
    assert stream == [5 if i % 2 else 3 for i in range(n)]


def test_unpack_records_order():
    from semantic_segmentation_server_amd.parallel.dp import unpack_records
    K = 3
    packed = np.zeros((2, 1 + 5 * K), np.float32)
    packed[0, 0] = 2
    packed[0, 1:11] = [7, 1, 0.1, 0.2, 0.3, 15, 0.5, 0.2, 0.3, 0.4]
    packed[1, 0] = 0
    r = unpack_records(packed, K, [5, 6], [1.0, 2.0], [0, 1])
    assert r["label"].tolist() == [7, 15] and r["frame"].tolist() == [5, 5]


def test_unpack_records_pool_exhausted():
    """A NaN count (the device root pool overflowed for that frame) gives no records and is
    counted, the other frames unpack as usual."""
    from semantic_segmentation_server_amd.parallel import dp
    K = 2
    packed = np.zeros((3, 1 + 5 * K), np.float32)
    packed[0, 0] = np.nan
    packed[1, 0] = 1
    packed[1, 1:6] = [9, 1, 0.1, 0.2, 0.3]
    packed[2, 0] = -2
    before = dp.pool_exhausted_frames()
    r = dp.unpack_records(packed, K, [1, 2, 3], [0.0] * 3, [0] * 3)
    assert r["frame"].tolist() == [2, 3, 3] and r["label"][0] == 9
    assert dp.pool_exhausted_frames() == before + 1


def _serve_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import grpc
    from semantic_segmentation_server_amd import config as C
    from semantic_segmentation_server_amd.api import proto as P
    from semantic_segmentation_server_amd.api.service import SemanticSegmentationStub, SemanticSegmentationV2Stub
    from semantic_segmentation_server_amd.parallel import dist as D
    from semantic_segmentation_server_amd.parallel.serving import DistributedServer
    ctx = D.init("gloo")
    cfg = C.parse(["--port", "0", "--host", "127.0.0.1", "--device", "cpu", "--input_size", "65",
                   "--batch", "2", "--streams", "2", "--gpus", str(world)])
    srv = DistributedServer(cfg, ctx, max_steps=3)
    srv.run()
    D.barrier(ctx)
    if ctx.is_root:
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            d = SemanticSegmentationStub(ch).GetSegmentedObjects(P.Empty())
            v2 = SemanticSegmentationV2Stub(ch)
            ls = v2.ListStreams(P.Empty())
            h = v2.Health(P.Empty())
        q.put((len(d.data), [s.stream_id for s in ls.streams], h.world_size, srv.steps,
               srv.metrics.snapshot()["frames"]))
    srv.stop()
    D.destroy(ctx)


def test_distributed_server_cpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_serve_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    n, streams, world, steps, frames = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert n == 3 and streams == [0, 1, 2, 3] and world == 2 and steps == 3 and frames == 12


def _degrade_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import grpc
    from semantic_segmentation_server_amd import config as C
    from semantic_segmentation_server_amd.api import proto as P
    from semantic_segmentation_server_amd.api.service import HealthStub, SemanticSegmentationV2Stub
    from semantic_segmentation_server_amd.parallel import dist as D
    from semantic_segmentation_server_amd.parallel.serving import DistributedServer
    ctx = D.init("gloo", timeout_s=60)
    cfg = C.parse(["--port", "0", "--host", "127.0.0.1", "--device", "cpu", "--input_size", "65",
                   "--batch", "2", "--streams", "1", "--gpus", str(world),
                   "--inject_fault", "1:2", "--rank_timeout", "60"])
    srv = DistributedServer(cfg, ctx, max_steps=6)
    try:
        srv.run()
    except RuntimeError:
        if rank == 1:
            os._exit(0)  # the lost rank: drop its connections abruptly
        raise
    with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
        h = SemanticSegmentationV2Stub(ch).Health(P.Empty())
        g = HealthStub(ch).Check(P.HealthCheckRequest())
    q.put((srv.steps, srv.degraded, h.ranks_alive, h.world_size, h.detail, g.status,
           srv.metrics.snapshot()["frames"]))
    srv.stop()


def test_rank_loss_degrades_to_rank0():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_degrade_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    steps, degraded, alive, world, detail, status, frames = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert degraded and steps == 6 and alive == 1 and world == 2 and "degraded" in detail
    assert status == 1  # SERVING
    # 2 lock-step steps on 2 ranks (4 frames each), then 4 steps on rank 0 alone (2 frames each)
    assert frames == 2 * 4 + 4 * 2


def _reform_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import grpc
    from semantic_segmentation_server_amd import config as C
    from semantic_segmentation_server_amd.api import proto as P
    from semantic_segmentation_server_amd.api.service import SemanticSegmentationV2Stub
    from semantic_segmentation_server_amd.parallel import dist as D
    from semantic_segmentation_server_amd.parallel.serving import DistributedServer
    ctx = D.init("gloo", timeout_s=60)
    cfg = C.parse(["--port", "0", "--host", "127.0.0.1", "--device", "cpu", "--input_size", "65",
                   "--batch", "2", "--streams", "1", "--gpus", str(world), "--min_area_ratio", "0",
                   "--inject_fault", "2:2", "--rank_timeout", "60"])
    srv = DistributedServer(cfg, ctx, max_steps=6)
    try:
        srv.run()
    except RuntimeError:
        if ctx.orig_rank == 2:
            os._exit(0)  # the lost rank: drop its connections abruptly
        raise
    out = (srv.ctx.orig_rank, srv.steps, srv.run_ctx.world, srv.run_ctx.members)
    if srv.ctx.is_root:
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            h = SemanticSegmentationV2Stub(ch).Health(P.Empty())
        per_stream = {s: b.pushed for s, b in srv.hub.buffers.items()}
        out = out + (h.ranks_alive, h.world_size, h.detail, srv.metrics.snapshot()["frames"], per_stream)
    q.put(out)
    srv.stop()
    D.destroy(srv.run_ctx)


def test_rank_loss_reshards_to_survivors():
    """World 3, launch rank 2 dies at step 2: ranks 0 and 1 re-form a 2-rank group and
    both keep serving their own streams (SURVEY.md §5.3 P-1 re-shard)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reform_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted((q.get(timeout=300) for _ in range(2)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0, r1 = got
    assert r0[:4] == (0, 6, 2, [0, 1]) and r1[:4] == (1, 6, 2, [0, 1])
    alive, wsize, detail, frames, per_stream = r0[4:]
    assert alive == 2 and wsize == 3 and "degraded to 2/3" in detail
    # 2 steps x 3 ranks x 2 frames, then 4 steps x 2 ranks x 2 frames
    assert frames == 2 * 6 + 4 * 4
    assert per_stream[1] > 0 and per_stream[0] > 0   # rank 1's camera still served after the loss


def _gather_timing_worker(rank, world, port, q, iters):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import time
    import torch.distributed as dist
    from semantic_segmentation_server_amd.parallel import dist as D
    ctx = D.init("gloo")
    K = 64
    rec = torch.zeros((32, 1 + 5 * K), dtype=torch.float32)   # one rank's step: 32 frames, 41 KB
    land = [torch.empty_like(rec) for _ in range(world)] if ctx.is_root else None
    ts = []
    for it in range(iters):
        D.barrier(ctx)
        t0 = time.perf_counter()
        dist.gather(rec, land, dst=0, group=ctx.cpu_group)
        ts.append(time.perf_counter() - t0)
    if ctx.is_root:
        q.put(sorted(ts))
    D.destroy(ctx)


def test_gloo_record_gather_cost_world8():
    """The default multi-GPU record path is a host gloo gather of every rank's packed
    records (32 frames x 1.3 KB = 41 KB) to rank 0, once per step on the collecting
    thread. At world size 8 it must stay far below the ~1.3 ms step it overlaps
    (VERDICT r1 4c): measured here with 8 CPU processes on loopback."""
    world, iters = 8, 60
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_timing_worker, args=(r, world, port, q, iters))
             for r in range(world)]
    for p in procs:
        p.start()
    ts = q.get(timeout=240)
    for p in procs:
        p.join(60)
    p50, p90 = ts[len(ts) // 2], ts[int(len(ts) * 0.9)]
    print(f"gloo gather world 8, 41 KB/rank: p50 {p50 * 1e3:.3f} ms p90 {p90 * 1e3:.3f} ms")
    # with a core per rank and its gloo threads (an MI355X node; the 16-CPU GPU box
    # measured p50 0.295 ms, profiles/r2_pg_ab.txt) the gather is a fifth of the step;
    # an 8-CPU container running 8 busy ranks is contention-bound (p50 ~2 ms alone, 10.4 ms
    # next to other test workers under pytest -n 4), so there only a sanity bound applies
    bound = 0.7e-3 if (os.cpu_count() or 1) >= 2 * world else 25e-3
    assert p50 < bound, p50


def test_rccl_uid_bytes_roundtrip_with_nuls():
    """an ncclUniqueId holds NUL bytes (magic, then a sockaddr whose
    family field is 02 00); reading or assigning the c_char field truncates at the first
    NUL. The raw-bytes path must keep all 128 bytes."""
    from semantic_segmentation_server_amd.parallel import rccl
    raw = bytes([0x4e, 0x43, 0, 0, 0x12, 0, 0, 0, 2, 0, 0x75, 0x31, 127, 0, 0, 1]) + \
        bytes((i * 37) % 256 for i in range(112))
    uid = rccl.uid_from_bytes(raw)
    assert rccl.uid_bytes(uid) == raw
    assert len(bytes(uid.internal)) < len(raw)  # the truncating accessor this path avoids
    with pytest.raises(ValueError):
        rccl.uid_from_bytes(raw[:64])


def _uid_worker(rank, world, port, raw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from semantic_segmentation_server_amd.parallel import dist as D
    from semantic_segmentation_server_amd.parallel import rccl
    ctx = D.init("gloo")
    uid = rccl.uid_from_bytes(raw) if rank == 0 else rccl._UniqueId()
    got = rccl.share_uid(ctx, uid)
    q.put((rank, rccl.uid_bytes(got)))
    D.barrier(ctx)
    D.destroy(ctx)


def test_rccl_uid_broadcast_world3():
    """The id rank 0 made reaches every rank byte for byte over the host group."""
    raw = bytes([0, 0, 0, 0, 2, 0, 0x75, 0x31]) + bytes(range(1, 121))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uid_worker, args=(r, 3, port, raw, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(got[r] == raw for r in range(3))
