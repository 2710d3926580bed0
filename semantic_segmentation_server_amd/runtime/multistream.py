"""Concurrent camera streams on one GPU (BASELINE config 5).

``StreamGroup`` owns S engines on the same device. Each has its own HIP stream,
its own static buffers and its own captured hipGraph (weights are packed per
engine; MobileNetV2 weights are ~6 MB so duplication is immaterial on a 288 GB
part). A step splits the rank's frame batch into S per-stream chunks, replays the
S graphs concurrently on their streams (the GPU overlaps them: the per-stream
graphs are launch/latency-bound at small per-stream batches), and joins the
packed records back on the caller's stream. To the data-parallel pipeline it
looks like one engine (``run_device`` -> (None, packed records)).

The reference serves exactly one camera (sem_seg_server.py:144,256).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from ..config import Config
from .engine import Engine


class StreamGroup:
    def __init__(self, cfg: Config, device: torch.device, streams: int,
                 model: Optional[torch.nn.Module] = None):
        if streams < 1:
            raise ValueError("streams >= 1")
        self.cfg = cfg
        self.device = device
        self.is_cuda = device.type == "cuda"
        self.engines: List[Engine] = []
        for s in range(streams):
            # same seed -> identical random-init weights on every stream
            self.engines.append(Engine(cfg, device, model=model))
        self.streams = [e.stream for e in self.engines]
        self.backend = self.engines[0].backend
        self._out = {}

    @property
    def H(self):
        return self.engines[0].H

    @property
    def W(self):
        return self.engines[0].W

    def set_camera(self, cam_w: int, cam_h: int) -> None:
        for e in self.engines:
            e.set_camera(cam_w, cam_h)

    def bind_inputs(self, bufs, split_post: bool = False) -> None:
        """Bind each engine to its slice of the pipeline's staging slots (one graph per
        slot and stream reads its frames in place). ``split_post``: every engine's
        post-processing graph runs on that engine's result stream, overlapping the
        next step's models; the packed records of all streams are joined on this
        group's ``result_stream``."""
        if not self.is_cuda:
            return
        S = len(self.engines)
        # each split engine adds a second stream; HIP maps all streams of a process
        # onto GPU_MAX_HW_QUEUES (4) hardware queues, and 2 S + 1 streams sharing them
        # serialise behind each other (measured: 4 streams x 8 frames 11.8k -> 10.7k
        # fps with split on), so the split only applies while the streams fit
        split_post = bool(split_post) and 2 * S + 1 <= int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        for i, e in enumerate(self.engines):
            e.bind_inputs([b.chunk(S)[i] for b in bufs], split_post=split_post)
        self._split = bool(split_post) and all(getattr(e, "_split", False) for e in self.engines)
        self.result_stream = torch.cuda.Stream(self.device) if self._split else None
        self._copied = [torch.cuda.Event() for _ in self.engines] if self._split else None

    def run_device(self, frames: torch.Tensor):
        B = frames.shape[0]
        S = len(self.engines)
        if B % S:
            raise ValueError(f"batch {B} not divisible by {S} streams")
        chunks = frames.chunk(S)
        K = self.cfg.max_segments
        out = self._out.get(B)
        if out is None:
            out = self._out[B] = torch.zeros((B, 1 + 5 * K), dtype=torch.float32, device=self.device)
        if not self.is_cuda:
            for i, (e, c) in enumerate(zip(self.engines, chunks)):
                _, p = e.run_device(c)
                out[i * (B // S):(i + 1) * (B // S)].copy_(p)
            return None, out
        cur = torch.cuda.current_stream(self.device)
        n = B // S
        split = getattr(self, "_split", False)
        rs = self.result_stream if split else None
        for i, (e, st, c) in enumerate(zip(self.engines, self.streams, chunks)):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                _, p = e.run_device(c)
                if not split:
                    out[i * n:(i + 1) * n].copy_(p, non_blocking=True)
            if split:  # engine i's records appear on its result stream
                rs.wait_stream(e.result_stream)
                with torch.cuda.stream(rs):
                    out[i * n:(i + 1) * n].copy_(p, non_blocking=True)
                self._copied[i].record(rs)
                e.result_stream.wait_event(self._copied[i])  # its next post-processing rewrites p
        for st in self.streams:
            cur.wait_stream(st)  # the models are done with this step's frames
        return None, out

    def records_from_labels(self, labels, frame_ids, ts, streams):  # host fallback unused
        raise RuntimeError("StreamGroup requires device post-processing (contour_mode fast)")
