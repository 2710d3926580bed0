"""Process-group plumbing.

One process per GPU; ``torch.distributed`` with backend ``"nccl"``, which binds
RCCL on ROCm (xGMI between the GPUs of a node), or ``"gloo"`` on CPU for tests.
Rendezvous comes from the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT); MASTER_ADDR defaults to 127.0.0.1.

The reference has no distributed code at all (single Edge TPU, batch 1).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None
    cpu_group: Optional[object] = None  # gloo group for host-memory collectives (None: default group)

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    @property
    def initialized(self) -> bool:
        return self.backend is not None


def init(backend: Optional[str] = None, timeout_s: float = 300.0,
         device: str = "auto") -> DistContext:
    """Initialise from env. Single process (no WORLD_SIZE) -> no process group.

    ``device``: "auto" (the local GPU unless ``backend`` is gloo), "cuda" (the local
    GPU whatever the backend: a gloo group driving GPU ranks) or "cpu".
    ``backend`` (or env SSA_PG_BACKEND): "nccl" (RCCL) or "gloo". The GPU data path
    only needs RCCL for the frame scatter / device record gather; the default serving
    and bench path gathers host records over gloo (see DataParallelPipeline)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    backend = backend or os.environ.get("SSA_PG_BACKEND") or None
    if device == "auto":
        use_cuda = torch.cuda.is_available() and backend != "gloo"
    else:
        use_cuda = device == "cuda"
    if use_cuda:
        if os.environ.get("SSA_SHARE_GPU", "0") == "1":
            # rehearsal knob: several ranks on one GPU (a 1-GPU box running the
            # multi-rank bench / server path over a gloo group); RCCL refuses this
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world == 1 and os.environ.get("SSA_FORCE_PG", "0") != "1":
        return DistContext(0, 1, 0, device, None)
    # SSA_FORCE_PG=1: a real (world-size 1) process group, so the single-GPU box can
    # rehearse the collective path of the multi-GPU run (RCCL streams, gathers)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    backend = backend or ("nccl" if use_cuda else "gloo")
    kw = {}
    if backend == "nccl" and os.environ.get("SSA_NCCL_EAGER", "0") == "1":
        # eager communicator init. Off by default: HIP maps streams onto 4 hardware
        # queues in creation order, and RCCL's streams created before the engine's shift
        # the compute / result / copy streams onto a worse mapping (world-size-1 rehearsal:
        # 17.6k frames/s eager vs 21.4k lazy, where the first collective creates them)
        kw["device_id"] = device
    dist.init_process_group(backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    # host-memory collectives (the per-step record gather) go over gloo, so the step
    # loop never enqueues an RCCL kernel beside the compute graphs
    cpu_group = dist.new_group(backend="gloo") if backend == "nccl" else None
    return DistContext(rank, world, local, device, backend, cpu_group)


def barrier(ctx: DistContext) -> None:
    if ctx.initialized:
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


def allreduce_max(ctx: DistContext, v: float) -> float:
    if not ctx.initialized:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=ctx.device if ctx.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(ctx: DistContext, v: float) -> float:
    if not ctx.initialized:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=ctx.device if ctx.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def destroy(ctx: DistContext) -> None:
    if ctx.initialized and dist.is_initialized():
        dist.destroy_process_group()
