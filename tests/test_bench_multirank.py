"""The driver's multi-GPU command, rehearsed on the CPU (VERDICT r3 #3c).

The driver launches ``python -m torch.distributed.run --nnodes=1 --nproc-per-node N
--master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W`` on an
8-GPU node. The same command runs here over gloo with the torch backend at a small input:
the JSON line must come from rank 0 alone, count every rank, and the frames collected on
rank 0 must carry every rank's stream id with per-stream frame ids in order (one lost,
duplicated or overwritten metadata slot breaks that)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,ingest,gb", [(2, "local", 0), (3, "local", 0), (2, "scatter", 0),
                                              (2, "local", 4)])
def test_bench_torchrun_cpu(world, ingest, gb):
    """gb > 0: --global_batch (strong scaling, BASELINE config 3 as written): the node-wide
    batch is split over the ranks."""
    steps, warmup, batch = 3, 1, 2
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", SSA_NUMA_PIN="0",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", str(steps),
           "--warmup", str(warmup), "--backend", "torch", "--input_size", "129",
           "--rpc", "0", "--ingest", ingest] + (["--global_batch", str(gb)] if gb else ["--batch", str(batch)])
    if gb:
        batch = gb // world
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == world
    assert out["steps"] == steps and out["warmup"] == warmup
    assert out["config"]["global_batch"] == batch * world
    assert out["config"]["parallelism"] == f"dp{world}"
    assert out["scaling"] == ("strong" if gb else "weak")
    assert out["value"] > 0 and out["ms_per_step"] > 0
    # every rank's frames reached rank 0, tagged with their own stream, ids in order
    assert out["frames_collected"] == steps * batch * world
    assert out["streams_collected"] == list(range(world))
    assert out["frame_order_errors"] == 0
    assert out["p50_frame_latency_ms"] is not None and out["p50_frame_latency_ms"] > 0


def test_bench_gpus_without_launcher_cpu():
    """``python bench.py --gpus 3`` with no torchrun means three ranks: the
    parent starts them itself and prints rank 0's one JSON line."""
    world, steps, warmup, batch = 3, 3, 1, 2
    env = dict(os.environ, OMP_NUM_THREADS="1", SSA_NUMA_PIN="0", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", str(steps),
           "--warmup", str(warmup), "--backend", "torch", "--input_size", "129", "--rpc", "0",
           "--batch", str(batch)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["config"]["parallelism"] == f"dp{world}"
    assert out["frames_collected"] == steps * batch * world
    assert out["streams_collected"] == list(range(world))
    assert out["pg_backend"] == "gloo" and out["gather"] == "host" and out["rccl_nranks"] is None


def test_bench_world_size_mismatch_fails():
    """Under a launcher, --gpus must match WORLD_SIZE: a silent 1-rank run is an error."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1"],
                       cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_bench_rccl_gather_world1_reports_nranks():
    """The RCCL record-gather path on a real (world-size-1) RCCL group: the JSON proves how
    many ranks RCCL joined (ncclCommCount) and every frame still reaches the hub."""
    env = dict(os.environ, SSA_FORCE_PG="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    steps, batch = 4, 4
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", str(steps),
                        "--warmup", "2", "--batch", str(batch), "--rpc", "0", "--gather", "rccl"],
                       cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["rccl_nranks"] == 1 and out["pg_backend"] == "nccl" and out["gather"] == "rccl"
    assert out["frames_collected"] == steps * batch
