"""T5: config-1 plumbing — CPU engine + producer + gRPC loopback (no GPU)."""
import os
import time

import grpc
import numpy as np
import torch

from semantic_segmentation_server_amd import config as C
from semantic_segmentation_server_amd.api import proto as P
from semantic_segmentation_server_amd.api.service import SemanticSegmentationStub, SemanticSegmentationV2Stub
from semantic_segmentation_server_amd.runtime.engine import Engine
from semantic_segmentation_server_amd.server import Server


def test_server_end_to_end_cpu():
    cfg = C.parse(["--port", "0", "--device", "cpu", "--input_size", "65", "--batch", "2",
                   "--host", "127.0.0.1", "--streams", "2"])
    srv = Server(cfg, max_steps=3).start()
    try:
        srv.producer.join(timeout=120)
        assert srv.producer.steps == 3 and srv.producer.error is None
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            st = SemanticSegmentationStub(ch)
            assert st.GetCameraResolution(P.Empty()).width == 640
            assert len(st.GetSegmentedObjects(P.Empty()).data) == 3
            v2 = SemanticSegmentationV2Stub(ch)
            assert v2.GetStats(P.Empty()).frames == 6
            assert len(v2.ListStreams(P.Empty()).streams) == 2
    finally:
        srv.stop(0)


class _PlantedEngine(Engine):
    """CPU engine whose 'model' returns a planted label map (person blob)."""

    def _infer_eager(self, frames):
        B = frames.shape[0]
        lab = torch.zeros(B, self.H, self.W, dtype=torch.uint8)
        lab[:, 20:50, 10:40] = 15
        lab[:, 60:90, 70:110] = 7
        return lab


def test_records_flow_into_rpc_newest_first():
    cfg = C.parse(["--port", "0", "--device", "cpu", "--input_size", "129", "--host", "127.0.0.1",
                   "--min_area_ratio", "0.01", "--camera_width", "129", "--camera_height", "129"])
    eng = _PlantedEngine(cfg)
    srv = Server(cfg, engine=eng, max_steps=2).start()
    try:
        srv.producer.join(timeout=60)
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            d = SemanticSegmentationStub(ch).GetSegmentedObjects(P.Empty())
        labels = [x.label for x in d.data]
        # each frame pushes [car (found later in raster pre-order first?), ...]; newest frame first
        assert set(labels) == {"person", "car"}
        assert all(0 < x.area <= 1 and 0 <= x.centroid.cx <= 1 for x in d.data)
        assert srv.hub.depth == 4 - 3 + 0  # 2 frames x 2 objects pushed, 3 popped
    finally:
        srv.stop(0)


def test_exact_and_fast_contour_modes_agree_cpu():
    cfg = C.parse(["--device", "cpu", "--input_size", "129", "--min_area_ratio", "0.01"])
    e_fast = _PlantedEngine(cfg)
    e_exact = _PlantedEngine(cfg.replace(contour_mode="exact"))
    f = np.zeros((1, 129, 129, 3), np.uint8)
    a = e_fast.step(f, [0], [0.0], 0)
    b = e_exact.step(f, [0], [0.0], 0)
    assert a.tolist() == b.tolist() and len(a) == 2


def test_debug_dump_writes_annotated_png(tmp_path):
    from PIL import Image
    from semantic_segmentation_server_amd import config as C
    from semantic_segmentation_server_amd.labels import load_labels, pascal_colormap
    from semantic_segmentation_server_amd.utils.debug_dump import render
    lab = np.zeros((129, 129), np.uint8)
    lab[20:80, 30:100] = 15
    lab[40:60, 50:70] = 0
    frame = np.full((96, 128, 3), 90, np.uint8)
    im = render(frame, lab, 129, 96, pascal_colormap(), load_labels(), min_area=50.0)
    assert im.size == (129, 96)
    a = np.asarray(im)
    assert (a == [0, 255, 0]).all(-1).sum() > 100      # contour outlines drawn
    assert (a == [255, 0, 0]).all(-1).sum() > 4        # centroid marker
    # engine hook: --debug_dump / --debug_every on the CPU path
    import torch
    from semantic_segmentation_server_amd.runtime.engine import Engine
    cfg = C.parse(["--device", "cpu", "--input_size", "65", "--debug_dump", str(tmp_path),
                   "--debug_every", "1"])
    e = Engine(cfg, torch.device("cpu"))
    e.step(np.full((1, 48, 64, 3), 128, np.uint8), [7], [0.0], 3)
    files = sorted(p.name for p in tmp_path.iterdir())
    assert files == ["s003_f00000007.png"]
    assert Image.open(tmp_path / files[0]).size[0] > 0


def test_debug_sync_sets_launch_blocking_and_disables_graphs(monkeypatch):
    """--debug_sync: HIP_LAUNCH_BLOCKING=1 before runtime init, eager launches."""
    from semantic_segmentation_server_amd import config as C
    monkeypatch.delenv("HIP_LAUNCH_BLOCKING", raising=False)
    cfg = C.apply_debug_env(C.parse([]))
    assert cfg.graph and "HIP_LAUNCH_BLOCKING" not in os.environ
    cfg = C.apply_debug_env(C.parse(["--debug_sync"]))
    assert cfg.debug_sync and not cfg.graph
    assert os.environ["HIP_LAUNCH_BLOCKING"] == "1"


def test_reservoir_add_many_and_frame_order_bookkeeping():
    """The vectorised per-step bookkeeping (Reservoir.add_many, DataParallelPipeline._observe)
    equals the per-sample loop it replaced: same ring contents, same frame-order verdicts."""
    import numpy as np
    from semantic_segmentation_server_amd.parallel.dp import DataParallelPipeline
    from semantic_segmentation_server_amd.utils.metrics import Reservoir
    vals = np.random.default_rng(0).random(29)
    a, b = Reservoir(8), Reservoir(8)
    for chunk in (vals[:3], vals[3:20], vals[20:]):
        for v in chunk:
            a.add(float(v))
        b.add_many(chunk)
        assert a.n == b.n and np.array_equal(a.buf, b.buf)

    class P:  # the attributes _observe touches
        frame_latency, metrics = Reservoir(64), None
        stream_last_id, stream_frames, frame_order_errors = {}, {}, 0
    p = P()
    # stream 0 in order, stream 1 with one repeat and one step back
    fids = [0, 10, 1, 11, 2, 11, 3, 9]
    sts = [0, 1, 0, 1, 0, 1, 0, 1]
    meta = np.stack([np.array(fids, np.float64), np.array(sts, np.float64), np.full(8, 1.0)], 1)
    DataParallelPipeline._observe(p, meta[:4])
    DataParallelPipeline._observe(p, meta[4:])
    assert p.frame_order_errors == 2
    assert p.stream_frames == {0: 4, 1: 4} and p.stream_last_id == {0: 3, 1: 9}
    assert p.frame_latency.n == 8
    # the plain-Python path (batches of <= 8 frames) and the vectorised one agree
    big = np.concatenate([meta] * 3)
    big[:, 0] += np.repeat([0, 100, 200], 8)

    def fresh():
        q = P()
        q.frame_latency, q.stream_last_id, q.stream_frames, q.frame_order_errors = Reservoir(64), {}, {}, 0
        return q
    q1, q2 = fresh(), fresh()
    DataParallelPipeline._observe(q1, big)          # 24 frames: numpy
    for k in range(0, 24, 8):
        DataParallelPipeline._observe(q2, big[k:k + 8])  # 8 at a time: plain Python
    assert (q1.frame_order_errors, q1.stream_frames, q1.stream_last_id) == \
        (q2.frame_order_errors, q2.stream_frames, q2.stream_last_id)
