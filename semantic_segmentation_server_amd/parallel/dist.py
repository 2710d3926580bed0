"""Process-group plumbing.

One process per GPU; ``torch.distributed`` with backend ``"nccl"``, which binds
RCCL on ROCm (xGMI between the GPUs of a node), or ``"gloo"`` on CPU for tests.
Rendezvous comes from the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT); MASTER_ADDR defaults to 127.0.0.1.

The reference has no distributed code at all (single Edge TPU, batch 1).
"""
from __future__ import annotations

import datetime
import logging
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

_log = logging.getLogger(__name__)


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None
    cpu_group: Optional[object] = None  # gloo group for host-memory collectives (None: default group)
    # elastic membership (reform()): the launch-time rank of every member of the current
    # group (index = current rank), the membership generation and the store that
    # survives a broken process group (hosted by launch rank 0)
    members: Optional[List[int]] = None
    gen: int = 0
    store: Optional[object] = None

    @property
    def orig_rank(self) -> int:
        return self.members[self.rank] if self.members else self.rank

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
    ``backend`` (or env SSA_PG_BACKEND): "nccl" (RCCL) or "gloo". With RCCL a gloo
    ``cpu_group`` is created beside it for host-side control traffic (heartbeat, pick
    broadcast, metadata, the default host record gather); the frame scatter and the
    opt-in device record gather go over RCCL (DataParallelPipeline)."""
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
    timeout = datetime.timedelta(seconds=timeout_s)
    # membership store for elastic re-forming after a rank loss: a TCPStore of its own
    # (MASTER_PORT + 1, or SSA_ELASTIC_PORT), hosted by launch rank 0, so it outlives a
    # broken process group (the PG's own store may belong to a torchrun agent)
    store = None
    if world > 1 and os.environ.get("SSA_ELASTIC", "1") != "0":
        port = int(os.environ.get("SSA_ELASTIC_PORT", int(os.environ["MASTER_PORT"]) + 1))
        store = dist.TCPStore(os.environ["MASTER_ADDR"], port, world, rank == 0, timeout=timeout,
                              wait_for_workers=False)
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=timeout, **kw)
    # host-memory control collectives (heartbeat, picks, metadata) go over gloo
    cpu_group = dist.new_group(backend="gloo") if backend == "nccl" else None
    return DistContext(rank, world, local, device, backend, cpu_group, list(range(world)), 0, store)


_graveyard: List[object] = []


def _drop_broken_group() -> None:
    """Unregister a process group whose peer is gone so a new one can be initialised.
    ``destroy_process_group`` (and a gloo ``abort``, measured: 60 s on a rank blocked in
    the heartbeat) waits for the pending collective to reach the group timeout; here the
    c10d registry is cleared at once and the old groups are aborted on a daemon thread
    (their sockets close when that returns; nothing waits on their pending work)."""
    if not dist.is_initialized():
        return
    import threading
    from torch.distributed import distributed_c10d as c10d
    w = c10d._world
    old = list(w.pg_names.keys())
    try:
        c10d._update_default_pg(None)
        for m in (w.pg_map, w.pg_names, w.pg_group_ranks, w.pg_backend_config, w.pg_to_tag,
                  w.tags_to_pg, w.pg_coalesce_state):
            m.clear()
        c10d._unregister_all_process_groups()
        w.group_count = 0
    except Exception as e:  # a torch without these internals: slow path
        _log.warning("reform: fast unregister failed (%r); destroying the group", e)
        try:
            dist.destroy_process_group()
        except Exception:
            pass
        return

    # keep the old groups referenced: their destructors join worker threads that are
    # blocked in the dead collective until the group timeout
    _graveyard.extend(old)

    def _abort(pgs):
        for pg in pgs:
            try:
                pg.abort()
            except Exception:
                pass
    threading.Thread(target=_abort, args=(old,), name="pg-abort", daemon=True).start()


def reform(ctx: DistContext, settle_s: float = 2.0, timeout_s: float = 60.0) -> DistContext:
    """Re-form the process group from the ranks still alive after a collective failed
    (fall back to P-1 ranks). Every survivor calls this; launch rank 0
    (the store host) waits until no new survivor has checked in for ``settle_s``, then
    publishes the member list of the next generation; the survivors renumber by launch
    rank and initialise a new group in a store namespace of that generation. Launch
    rank 0 must be among the survivors (it hosts the store and the RPC); the others
    raise if it is gone. Reference: the reference simply exits with its producer
    (/root/reference/sem_seg_server.py:286-288)."""
    import time
    if ctx.store is None:
        raise RuntimeError("reform: no elastic store (world size 1 or SSA_ELASTIC=0)")
    store = ctx.store
    store.set(_abort_key(ctx), "1")  # wake peers blocked in this generation's heartbeat
    # membership waits outlast a peer's failure detection (up to one PG timeout)
    store.set_timeout(datetime.timedelta(seconds=2 * timeout_s + settle_s))
    t0 = time.time()
    _drop_broken_group()
    _log.info("reform: dropped the broken group in %.2f s", time.time() - t0)
    gen = ctx.gen + 1
    me = ctx.orig_rank
    key = f"ssa/gen{gen}"
    store.set(f"{key}/alive/{me}", "1")
    n = store.add(f"{key}/count", 1)
    if me == 0:
        last, t_last, t0 = n, time.time(), time.time()
        while time.time() - t_last < settle_s and time.time() - t0 < timeout_s:
            time.sleep(0.05)
            cur = store.add(f"{key}/count", 0)
            if cur != last:
                last, t_last = cur, time.time()
            if cur >= len(ctx.members or [0]):
                break
        alive = sorted(r for r in (ctx.members or [0]) if r == 0 or store.check([f"{key}/alive/{r}"]))
        store.set(f"{key}/members", ",".join(str(r) for r in alive))
    members = [int(v) for v in store.get(f"{key}/members").decode().split(",")]
    if me not in members:
        raise RuntimeError(f"reform: launch rank {me} checked in too late for generation {gen}")
    _log.info("reform: members %s agreed after %.2f s", members, time.time() - t0)
    rank, world = members.index(me), len(members)
    pg_store = dist.PrefixStore(f"{key}/pg", store)
    backend = ctx.backend or "gloo"
    dist.init_process_group(backend, store=pg_store, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s))
    cpu_group = dist.new_group(backend="gloo") if backend == "nccl" else None
    return DistContext(rank, world, ctx.local_rank, ctx.device, backend, cpu_group, members, gen, store)


def barrier(ctx: DistContext) -> None:
    """Host barrier over the gloo group (beside an RCCL default group too): it orders
    the ranks' host threads, which is all the callers need (they synchronise their own
    device around it), and it never makes torch create a ProcessGroupNCCL communicator
    of its own next to the pipeline's stream-ordered ones (parallel/rccl.py)."""
    if ctx.initialized:
        dist.barrier(group=ctx.cpu_group)


class PeerLost(RuntimeError):
    pass


def _abort_key(ctx: DistContext) -> str:
    return f"ssa/gen{ctx.gen}/abort"


def allreduce_max(ctx: DistContext, v: float, poll_s: float = 0.05) -> float:
    """Max over ranks (the per-step stop flag, i.e. the heartbeat of the serving loop).

    With an elastic store the all-reduce is asynchronous and polled: a survivor that saw
    a peer fail posts an abort key for the current generation, and every rank blocked in
    this heartbeat raises ``PeerLost`` within ``poll_s`` instead of sitting out the
    process-group timeout (in a gloo ring only the failed rank's neighbours see the
    connection drop)."""
    if not ctx.initialized:
        return v
    # host flag over the gloo group (the CPU group beside an RCCL default group): the
    # heartbeat never puts an RCCL kernel or a device sync into the step loop
    t = torch.tensor([v], dtype=torch.float64)
    grp = ctx.cpu_group
    if ctx.store is None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=grp)
        return float(t.item())
    import time
    work = dist.all_reduce(t, op=dist.ReduceOp.MAX, async_op=True, group=grp)
    t_next = time.perf_counter() + poll_s
    while not work.is_completed():
        now = time.perf_counter()
        if now >= t_next:
            t_next = now + poll_s
            if ctx.store.check([_abort_key(ctx)]):
                raise PeerLost(f"generation {ctx.gen} aborted by a peer")
        time.sleep(1e-5)
    work.wait()  # surfaces a failed collective as an exception
    return float(t.item())


def broadcast_obj(ctx: DistContext, obj):
    """Rank 0's picklable ``obj`` on every rank (host group: gloo when RCCL is the
    default backend). Used once per plan build to share rank 0's autotune picks."""
    if ctx.world == 1 or not ctx.initialized:
        return obj
    buf = [obj if ctx.is_root else None]
    dist.broadcast_object_list(buf, src=0, group=ctx.cpu_group)
    return buf[0]


def allreduce_sum(ctx: DistContext, v: float) -> float:
    if not ctx.initialized:
        return v
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=ctx.cpu_group)
    return float(t.item())


def destroy(ctx: DistContext) -> None:
    if ctx.initialized and dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:  # a broken group (peer lost) may fail its own teardown
            pass
