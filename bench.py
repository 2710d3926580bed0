#!/usr/bin/env python3
"""Headline benchmark: frames/sec (whole node) + p50 GetSegmentedObjects latency.

Config (BASELINE.json): DeepLabv3-MobileNetV2, 513x513, PASCAL VOC (21 classes),
bf16, synthetic 640x480 BGR camera frames, random-init weights. One process per
GPU (torchrun); per-rank batch ``--batch`` (default 32) => weak scaling; ``--global_batch G``
=> strong scaling (G / N frames per rank, BASELINE config 3 as written: 32 over 8 GPUs).

One timed step, on every rank:
  H2D of the rank's next frames (pinned, copy stream, overlapped) or the rank-0
  upload + RCCL scatter (``--ingest scatter``)
  -> hipGraph replay: letterbox/normalise + DeepLabv3 + upsample/argmax + mask +
     CCL + contour statistics -> packed records
  -> records + frame metadata to rank 0 (pinned host memory over gloo by default, one step
     late; ``--gather rccl``: an RCCL gather of a packed device row) -> push into the
     LIFO result hub.

After the timed region, rank 0 serves the hub over gRPC on loopback and a client
subprocess measures GetSegmentedObjects latency while all ranks keep stepping
(the RPC is served under inference load, as in production).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...

``--gpus N`` means N ranks in both launch forms: under torchrun it must equal WORLD_SIZE
(else exit 2); without a launcher this process (which never touches the GPU) starts N
rank processes itself, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT set before any GPU call, and rank 0's JSON line is the output. At N > 1 on
GPUs the records reach rank 0 through the stream-ordered RCCL gather (parallel/rccl.py);
the JSON reports ``rccl_nranks`` from ``ncclCommCount`` on rank 0's communicator.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

BASELINE_METRIC = "frames/sec (whole node) + p50 GetSegmentedObjects latency, 513x513 PASCAL VOC"


def _client_proc(port: int, n: int, conn) -> None:
    try:
        from semantic_segmentation_server_amd.client import rpc_latency
        conn.send(rpc_latency(f"127.0.0.1:{port}", n=n, warmup=min(200, n)))
    except Exception as e:  # pragma: no cover
        conn.send({"error": repr(e)})
    conn.close()


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch", type=int, default=32, help="frames per GPU per step")
    p.add_argument("--backend", choices=["hip", "torch"], default="hip")
    p.add_argument("--lag", type=int, default=2, choices=[0, 1, 2],
                   help="pipeline lag (2 = three steps in flight, the throughput default; "
                        "0 = one step in flight, records collected synchronously: the "
                        "latency configuration)")
    p.add_argument("--arch", default="mnv2")
    p.add_argument("--aspp", default="full")
    p.add_argument("--input_size", type=int, default=513)
    p.add_argument("--camera", default="640x480")
    p.add_argument("--ingest", choices=["local", "scatter"], default="local",
                   help="local: each rank uploads its own frames (the default); scatter: rank 0 "
                        "uploads the node batch and ncclScatter spreads it (an ablation: at N = 8, "
                        "B = 32 rank 0's one PCIe link carries 256 x 921.6 KB = 236 MB per step, "
                        "~4.3 ms at ~55 GB/s against a ~0.9 ms step)")
    p.add_argument("--gather", choices=["auto", "host", "rccl"], default="auto",
                   help="record gather to rank 0: rccl = ncclGather of packed record rows over "
                        "xGMI, enqueued on the result stream (the auto choice on GPUs at N > 1); "
                        "host = each rank's records written to pinned memory by a kernel and "
                        "gathered over gloo (the auto choice at N = 1 and on CPU; an ablation at "
                        "N > 1). World-size-1 cost of the RCCL gather: 1.2-2.5 %% "
                        "(profiles/r5f_rccl_world1_ab.txt)")
    p.add_argument("--pg", choices=["auto", "nccl", "gloo"], default="auto",
                   help="process-group backend; auto: RCCL (+ a gloo control group) when an "
                        "RCCL data path is in use (--ingest scatter, the RCCL gather), else gloo")
    p.add_argument("--contour_mode", choices=["fast", "exact", "none"], default="fast")
    p.add_argument("--no-graph", dest="graph", action="store_false")
    p.add_argument("--rpc", type=int, default=2000, help="GetSegmentedObjects calls to time (0: skip)")
    p.add_argument("--dtype", default="bf16")
    p.add_argument("--streams", type=int, default=1,
                   help="concurrent camera streams per GPU: their frames fill one batched step "
                        "(one hipGraph; records tagged with their stream id)")
    p.add_argument("--per_stream_graphs", action="store_true",
                   help="config-5 alternative: one engine + HIP stream + hipGraph per camera "
                        "stream (measured slower than the batched step, kept for comparison)")
    p.add_argument("--serve", action="store_true",
                   help="time the real serving loop (Server / DistributedServer: feeder thread, "
                        "pinned ring, lag-1 pipeline, gRPC services up) instead of the bench loop")
    p.add_argument("--supervise", action="store_true",
                   help="with --serve: the CLI default -- a parent that never touches the GPU hosts "
                        "gRPC + hub, --gpus worker processes run the pipeline and ship records "
                        "through shared-memory rings (runtime/supervisor.py)")
    p.add_argument("--global_batch", type=int, default=0,
                   help="strong scaling: a fixed node-wide batch split over the ranks (per-GPU "
                        "batch = global_batch / N; BASELINE config 3 as written: 32 over 8 GPUs)")
    a = p.parse_args()
    if a.gpus < 1:
        p.error("--gpus must be >= 1")
    if not a.supervise:
        ws = os.environ.get("WORLD_SIZE")
        if ws is not None and int(ws) != a.gpus:
            print(f"bench: --gpus {a.gpus} but the launcher started WORLD_SIZE={ws} ranks",
                  file=sys.stderr)
            return 2
        if ws is None and a.gpus > 1:
            return _spawn_ranks(a.gpus)
    a.scaling = "weak"
    if a.global_batch:
        nw = int(os.environ.get("WORLD_SIZE", "1")) if not a.supervise else max(1, a.gpus)
        if a.global_batch % nw:
            p.error(f"--global_batch {a.global_batch} is not a multiple of the {nw} ranks")
        a.batch = a.global_batch // nw
        a.scaling = "strong"
    if a.serve:
        return _serve_bench(a)
    # each rank's host threads and pinned staging on its GPU's NUMA node, before the first
    # GPU call of the process (VERDICT r3 #3b; serving does the same in serve_distributed)
    from semantic_segmentation_server_amd.parallel.affinity import pin_to_gpu_numa
    pin_to_gpu_numa()

    import numpy as np
    import torch
    from semantic_segmentation_server_amd import config as C
    from semantic_segmentation_server_amd.parallel import dist as D
    from semantic_segmentation_server_amd.parallel.dp import DataParallelPipeline
    from semantic_segmentation_server_amd.runtime.engine import Engine
    from semantic_segmentation_server_amd.runtime.results import ResultHub
    from semantic_segmentation_server_amd.runtime.sources import SyntheticSource

    import torch as _t
    world = int(os.environ.get("WORLD_SIZE", "1"))
    gpu = _t.cuda.is_available() and a.backend != "cpu"
    # SSA_SHARE_GPU=1 (rehearsal: several ranks on one GPU): RCCL refuses two ranks on one
    # device, so the auto choice is the gloo group with the host-memory gather
    share = os.environ.get("SSA_SHARE_GPU", "0") == "1"
    if share and a.ingest == "scatter":
        # the frame scatter is a device collective (gloo scatters CPU tensors only) and RCCL
        # refuses two ranks on one GPU: rehearse with local ingest instead
        print("bench: --ingest scatter needs RCCL, which SSA_SHARE_GPU=1 rules out; using local ingest",
              file=sys.stderr)
        a.ingest = "local"
    if a.gather == "auto":
        # N > 1 on GPUs: the records travel over xGMI (RCCL), as in the north-star config
        a.gather = "rccl" if (gpu and world > 1 and not share) else "host"
    pg = a.pg if a.pg != "auto" else (
        "nccl" if gpu and not share and (a.ingest == "scatter" or a.gather == "rccl") else "gloo")
    ctx = D.init(pg, device="cuda" if _t.cuda.is_available() and a.backend != "cpu" else "auto")
    cam_w, cam_h = (int(v) for v in a.camera.split("x"))
    cfg = C.Config(arch=a.arch, aspp=a.aspp, input_size=a.input_size, backend=a.backend,
                   dtype=a.dtype, batch=a.batch, graph=a.graph, contour_mode=a.contour_mode,
                   ingest=a.ingest, camera_width=cam_w, camera_height=cam_h,
                   num_classes=21 if a.arch == "mnv2" else 19,
                   dataset="pascal" if a.arch == "mnv2" else "cityscapes")
    if a.streams > 1 and a.per_stream_graphs:
        from semantic_segmentation_server_amd.runtime.multistream import StreamGroup
        engine = StreamGroup(cfg, ctx.device, a.streams)
    else:
        engine = Engine(cfg, ctx.device)
    hub = ResultHub(ctx.world * a.streams, maxlen=4096) if ctx.is_root else None
    # --lag L: step k collects step k-L's records, so the next graph launches and the host
    # unpack overlap the GPU instead of idling it; run_steps flushes the last steps inside
    # the timed region (every timed step's records reach the hub). Lag 2 (three steps in
    # flight on three slot-parallel plan copies, the serving default) is the default. Round
    # 2 kept lag 1 because short windows lost 20-45 % at lag 2; round 3 found the cause (a
    # D2H hipMemcpyAsync of the records blocking the host for ~6 ms every ~20 steps,
    # profiles/r3_lag_stall.txt) and writes the records to pinned memory with a kernel:
    # --steps 20 --warmup 5 now 29.8-29.9k frames/s at lag 2 vs 27.5-27.7k at lag 1.
    # synthetic camera frames, pinned; distinct per rank (prepared before the pipeline, whose
    # construction ends by priming its streams: the warmup then follows without a GPU-idle gap)
    src = SyntheticSource(cam_w, cam_h, stream=ctx.rank, seed=1, pool=max(2, min(a.batch, 8)))
    nb = a.batch * (ctx.world if (a.ingest == "scatter" and ctx.is_root) else 1)
    host_batches = []
    for k in range(2):
        frames, _, _ = src.read_batch(nb)
        host_batches.append(torch.from_numpy(np.ascontiguousarray(frames)).pin_memory()
                            if ctx.device.type == "cuda" else torch.from_numpy(frames.copy()))
    pipe = DataParallelPipeline(ctx, engine, cam_w, cam_h, a.batch, a.ingest, hub, a.streams,
                                lag=a.lag, gather=a.gather, auto_lag=False)

    verbose = os.environ.get("SSA_BENCH_VERBOSE", "0") == "1"

    staged = [False]  # the first batch of a run is already on its way (steady state)

    def run_steps(n: int, k0: int = 0, stage_next: bool = True) -> None:
        # double-buffered ingest: the next batch's H2D overlaps this step's compute;
        # the last step of a run stages the first batch of the next run
        if n <= 0:
            return
        if not staged[0]:
            pipe.prefetch(host_batches[k0 % 2])
        for k in range(n):
            last = k + 1 == n
            pipe.step(next_frames=host_batches[(k0 + k + 1) % 2] if (not last or stage_next) else None)
            if verbose:
                print(f"[rank {ctx.rank}] step {k0 + k} ok", file=sys.stderr, flush=True)
        pipe.flush()
        staged[0] = stage_next

    sync = (lambda: torch.cuda.synchronize(ctx.device)) if ctx.device.type == "cuda" else (lambda: None)
    t_w0 = time.perf_counter()
    run_steps(a.warmup)
    sync()
    warm_s = time.perf_counter() - t_w0
    D.barrier(ctx)
    sync()
    rec0, fr0 = pipe.records_out, pipe.frames_done
    pipe.reset_observations()
    w0, g0 = pipe.wait_s, pipe.gather_s
    t0 = time.perf_counter()
    run_steps(a.steps, a.warmup)
    t_host = time.perf_counter() - t0  # the host's step loop (the final sync excluded)
    sync()
    D.barrier(ctx)
    sync()
    dt = time.perf_counter() - t0
    # where rank 0's host thread spent the step loop: blocked on step-completion events,
    # in the host (gloo) record gather, or busy (launches, unpack, hub push)
    w_ms, g_ms = (pipe.wait_s - w0) / a.steps * 1e3, (pipe.gather_s - g0) / a.steps * 1e3
    host_ms = {"busy": round(t_host / a.steps * 1e3 - w_ms - g_ms, 4), "event_wait": round(w_ms, 4),
               "host_gather": round(g_ms, 4)}
    dt = D.allreduce_max(ctx, dt)

    frames_total = a.steps * a.batch * ctx.world
    fps = frames_total / dt
    # records that reached the hub from the timed steps (rank 0 collects every rank's)
    timed_records, timed_frames = pipe.records_out - rec0, pipe.frames_done - fr0
    # capture -> record-in-hub latency of the timed frames (rank 0 sees every rank's):
    # capture = the host batch handed to the pipeline (its H2D starts); with lag L, L + 1
    # steps are in flight, so this is ~(L + 1) step intervals plus the step's own time
    lat = pipe.frame_latency.values()
    frame_lat = {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99))} \
        if len(lat) else {"p50": None, "p99": None}
    streams_seen = sorted(int(k) for k in pipe.stream_frames)
    frames_collected = int(sum(pipe.stream_frames.values()))
    order_errors = int(pipe.frame_order_errors)

    rpc = None
    if a.rpc > 0:
        rpc = _rpc_under_load(ctx, pipe, hub, run_steps, a.rpc, D)

    if ctx.is_root:
        out = {
            "metric": _metric(a),
            "value": round(fps, 2),
            "unit": "frames/s",
            "n_gpus": ctx.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": f"synthetic {a.camera} BGR frames, random-init weights",
            "config": {
                "model": _model_name(a),
                "aspp": a.aspp,
                "global_batch": a.batch * ctx.world,
                "per_gpu_batch": a.batch,
                "seq_len": a.input_size,
                "input": f"{a.input_size}x{a.input_size}",
                "camera": a.camera,
                "classes": cfg.num_classes,
                "parallelism": f"dp{ctx.world}",
                "ingest": a.ingest,
                "gather": pipe.gather_mode,
                "process_group": ctx.backend,
                "rccl_nranks": pipe.rccl_nranks(),
                "backend": a.backend,
                "hipgraph": bool(a.graph and ctx.device.type == "cuda"),
                "contour_mode": a.contour_mode,
                "streams_per_gpu": a.streams,
                "stream_mode": "per-stream graphs" if (a.streams > 1 and a.per_stream_graphs)
                else "batched",
                "pipeline_lag": pipe.lag,
                "slot_parallel": bool(getattr(engine, "slot_parallel", False)),
            },
            "p50_get_segmented_objects_ms": rpc.get("p50_ms") if rpc else None,
            "p99_get_segmented_objects_ms": rpc.get("p99_ms") if rpc else None,
            "p50_frame_latency_ms": None if frame_lat["p50"] is None else round(frame_lat["p50"], 4),
            "p99_frame_latency_ms": None if frame_lat["p99"] is None else round(frame_lat["p99"], 4),
            "pg_backend": ctx.backend,
            "gather": pipe.gather_mode,
            "rccl_nranks": pipe.rccl_nranks(),
            "frames_collected": frames_collected,
            "streams_collected": streams_seen,
            "frame_order_errors": order_errors,
            "records_per_frame": round(timed_records / max(1, timed_frames), 4),
            "records_per_frame_under_rpc_load": (round(rpc["records"] / max(1, rpc["frames"]), 4)
                                                 if rpc and "records" in rpc else None),
            "warmup_s": round(warm_s, 2),
            "host_ms_per_step": host_ms,
        }
        print(json.dumps(out), flush=True)
    pipe.close()  # the pipeline's RCCL communicators, before the process group
    D.destroy(ctx)
    return 0


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn_ranks(n: int) -> int:
    """``python bench.py --gpus N`` without a launcher: start N rank processes of this
    same command (one per GPU), each with the torchrun environment set before it makes
    any GPU call; this parent imports no GPU library. Rank 0 prints the JSON line. The
    first rank to fail takes the others down (their exact PIDs) and sets the exit code."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    import signal

    def _stop(signum, _frame):  # a stopped parent takes its ranks down (exact PIDs)
        for q in procs:
            if q.poll() is None:
                q.terminate()
        raise SystemExit(128 + signum)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, _stop)
    rc = 0
    live = list(procs)
    while live:
        for pr in list(live):
            code = pr.poll()
            if code is None:
                continue
            live.remove(pr)
            if code != 0 and rc == 0:
                rc = code
                print(f"bench: rank {procs.index(pr)} exited with {code}; stopping the others",
                      file=sys.stderr)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


def _serve_bench(a) -> int:
    """Served fps: the production loop with a synthetic camera (no fps cap) and the
    gRPC services up; W steps of warmup, then the frames of the next K steps over their
    wall time, while a client subprocess times GetSegmentedObjects (rank 0)."""
    import threading
    import torch
    from semantic_segmentation_server_amd import config as C
    from semantic_segmentation_server_amd.parallel.affinity import pin_to_gpu_numa

    world = int(os.environ.get("WORLD_SIZE", "1"))
    pin_to_gpu_numa()
    cam_w, cam_h = (int(v) for v in a.camera.split("x"))
    cfg = C.Config(arch=a.arch, aspp=a.aspp, input_size=a.input_size, backend=a.backend,
                   dtype=a.dtype, batch=a.batch, graph=a.graph, contour_mode=a.contour_mode,
                   ingest=a.ingest, camera_width=cam_w, camera_height=cam_h, streams=a.streams,
                   num_classes=21 if a.arch == "mnv2" else 19, port=0, host="127.0.0.1",
                   dataset="pascal" if a.arch == "mnv2" else "cityscapes", gpus=world)
    total = a.warmup + a.steps
    sup = None
    if a.supervise:
        from semantic_segmentation_server_amd.runtime.supervisor import SupervisedServer
        world = max(1, a.gpus)
        cfg.gpus = world
        sup = srv = SupervisedServer(cfg).start()
        steps = lambda: sum(w.steps for w in sup.workers)  # noqa: E731
        root, port = True, srv.port
        t_up = time.time() + 900
        while not all(w.up for w in sup.workers) and time.time() < t_up and sup.alive:
            time.sleep(0.05)
        total = (a.warmup + a.steps) * world
    elif world > 1:
        from semantic_segmentation_server_amd.parallel import dist as D
        from semantic_segmentation_server_amd.parallel.serving import DistributedServer
        srv = DistributedServer(cfg, max_steps=None)
        ctx = srv.ctx
        steps = lambda: srv.steps  # noqa: E731
        stop_evt = threading.Event()
        th = threading.Thread(target=srv.run, args=(stop_evt,), daemon=True)
        root, port = ctx.is_root, None
        th.start()
    else:
        from semantic_segmentation_server_amd.server import Server
        srv = Server(cfg).start()
        steps = lambda: srv.producer.steps  # noqa: E731
        root, port = True, srv.port
    t_lim = time.time() + 600
    per = world if sup is not None else 1  # steps() counts every worker's steps
    while steps() < a.warmup * per and time.time() < t_lim:
        time.sleep(0.0005)
    if world > 1 and sup is None:
        port = srv.port
    s0, t0 = steps(), time.perf_counter()
    while steps() < s0 + a.steps * per and time.time() < t_lim:
        time.sleep(0.0002)
    s1, t1 = steps(), time.perf_counter()
    fps = (s1 - s0) * a.batch * (world // per) / (t1 - t0)
    s1, s0 = s0 + (s1 - s0) // per, s0
    rpc = None
    if root and a.rpc > 0 and port:
        mpctx = mp.get_context("spawn")
        parent, child = mpctx.Pipe()
        proc = mpctx.Process(target=_client_proc, args=(port, a.rpc, child), daemon=True)
        proc.start()
        rpc = parent.recv() if parent.poll(120) else {"error": "client timeout"}
        proc.join(10)
    extra = {}
    if sup is not None:
        snap = sup.metrics.snapshot()
        lat = snap.get("worker_frame_latency_ms") or snap.get("worker0_frame_latency_ms") or {}
        extra = {"p50_frame_latency_ms": lat.get("p50"), "p99_frame_latency_ms": lat.get("p99"),
                 "ipc_drops": snap.get("ipc_drops", 0), "worker_restarts": snap.get("worker_restarts", 0),
                 "records_pushed": int(sum(b.pushed for b in sup.hub.buffers.values()))}
        sup.stop(0)
    elif world > 1:
        stop_evt.set()
        th.join(60)
        srv.stop()
        D.destroy(srv.run_ctx)
    else:
        srv.stop(0)
    if root:
        out = {
            "metric": _metric(a), "value": round(fps, 2), "unit": "frames/s", "n_gpus": world,
            "steps": s1 - s0, "warmup": a.warmup, "ms_per_step": round((t1 - t0) / max(1, s1 - s0) * 1e3, 4),
            "higher_is_better": True, "scaling": a.scaling, "vs_baseline": None, "dtype": a.dtype,
            "data": f"synthetic {a.camera} BGR frames, random-init weights",
            "config": {"model": _model_name(a), "global_batch": a.batch * world, "seq_len": a.input_size,
                       "parallelism": f"dp{world}",
                       "mode": ("served, supervised workers (gRPC parent + per-GPU worker processes, "
                                "shared-memory record rings)" if sup is not None else
                                "served (feeder + lagged pipeline + gRPC)"),
                       "streams_per_gpu": a.streams},
            "p50_get_segmented_objects_ms": rpc.get("p50_ms") if rpc else None,
            "p99_get_segmented_objects_ms": rpc.get("p99_ms") if rpc else None,
        }
        out.update(extra)
        print(json.dumps(out), flush=True)
    return 0


def _model_name(a) -> str:
    return "DeepLabv3-MobileNetV2" if a.arch == "mnv2" else "DeepLabv3-ResNet50"


def _metric(a) -> str:
    """The headline metric string, with the config's own input size and dataset (the
    BASELINE.json string for the headline config)."""
    if a.arch == "mnv2" and a.input_size == 513:
        return BASELINE_METRIC
    ds = "PASCAL VOC" if a.arch == "mnv2" else "Cityscapes"
    return (f"frames/sec (whole node) + p50 GetSegmentedObjects latency, "
            f"{a.input_size}x{a.input_size} {ds}")


def _rpc_under_load(ctx, pipe, hub, run_steps, n_calls, D):
    """Rank 0 serves the hub; a client subprocess times GetSegmentedObjects while
    every rank keeps running pipeline steps. Returns the client's stats on rank 0."""
    import torch
    server = None
    parent = None
    proc = None
    if ctx.is_root:
        from semantic_segmentation_server_amd.api import service as S
        from semantic_segmentation_server_amd.labels import load_labels
        server, port = S.make_server(8, 0, "127.0.0.1")
        S.add_v1_servicer(S.SemanticSegmentationServicer(hub, load_labels(), 3, pipe.cam), server)
        server.start()
        mpctx = mp.get_context("spawn")
        parent, child = mpctx.Pipe()
        proc = mpctx.Process(target=_client_proc, args=(port, n_calls, child), daemon=True)
        proc.start()
    k = 0
    rec0, fr0 = pipe.records_out, pipe.frames_done
    t_end = time.time() + 120
    while True:
        done = 1.0 if (ctx.is_root and (parent.poll() or time.time() > t_end)) else 0.0
        if D.allreduce_max(ctx, done) > 0:
            break
        run_steps(1, k)
        k += 1
    res = None
    if ctx.is_root:
        res = parent.recv() if parent.poll(60) else {"error": "client timeout"}
        proc.join(10)
        server.stop(0)
        res["load_steps"] = k
        res["records"], res["frames"] = pipe.records_out - rec0, pipe.frames_done - fr0
    return res


if __name__ == "__main__":
    sys.exit(main())
