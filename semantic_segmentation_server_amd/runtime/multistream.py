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
        for i, (e, st, c) in enumerate(zip(self.engines, self.streams, chunks)):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                _, p = e.run_device(c)
                out[i * n:(i + 1) * n].copy_(p, non_blocking=True)
        for st in self.streams:
            cur.wait_stream(st)
        return None, out

    def records_from_labels(self, labels, frame_ids, ts, streams):  # host fallback unused
        raise RuntimeError("StreamGroup requires device post-processing (contour_mode fast)")
