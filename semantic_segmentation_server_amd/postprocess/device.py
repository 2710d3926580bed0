"""Device-side contour statistics (HIP kernels in ``csrc/hip/postprocess.hip``).

Static workspace + packed output per batch size so the whole thing replays
inside the engine's hipGraph; ``fetch`` does the single small D2H copy of the
packed records (1 + 5K floats per frame) and unpacks them in push order.
"""
from __future__ import annotations

import os

from typing import Dict, Sequence

import numpy as np
import torch

from ..ops import hip_ops
from ..runtime.results import RECORD_DTYPE


class DevicePostprocess:
    def __init__(self, device: torch.device, H: int, W: int, palette: np.ndarray, K: int = 64,
                 bins: int = 32, thr: int = 127):
        self.device = device
        self.H, self.W, self.K, self.bins, self.thr = H, W, K, bins, thr
        self.palette = torch.tensor(np.asarray(palette, np.int32).reshape(256, 3), device=device)
        self._bufs: Dict[int, tuple] = {}
        self._host: Dict[int, torch.Tensor] = {}
        # accumulation pass: pixel strips (0), LDS-staged 32 x 32 (1) or 64 x 64 (2) tiles;
        # unset: by batch size (accum_for)
        env = os.environ.get("SSA_POST_ACCUM")
        self.accum = int(env) if env is not None else None

    def accum_for(self, B: int) -> int:
        """The accumulation pass for a batch of B frames: the LDS-staged 32 x 32 tiles at every
        batch size since round 5's slot tables (batch 1: 18.6 vs 20.5 us for round 3's strips,
        5678 vs 5456 frames/s, p50 0.625 vs 0.638 ms, profiles/r6b_b1_accum_ab.txt; batch 32:
        64.8 vs 219 us per 32 bench frames, r5t). More than 32 classes use the strips (the
        tile kernel's dense class counters hold 32)."""
        if self.accum is not None:
            return self.accum
        return 1
    def _buffers(self, B: int):
        if B not in self._bufs:
            nbytes = hip_ops.post_workspace_bytes(B, self.H, self.W, self.K, self.bins)
            ws = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)  # deterministic start
            rec = torch.zeros((B, 1 + 5 * self.K), dtype=torch.float32, device=self.device)
            self._bufs[B] = (ws, rec)
        return self._bufs[B]

    def run(self, labels: torch.Tensor, crop_w: int, crop_h: int, min_area: float,
            out: torch.Tensor = None) -> torch.Tensor:
        """Packed records of ``labels`` into the static buffer for this B, or into ``out``
        ([B, 1 + 5K] fp32, e.g. a row slice of a bigger batch's buffer). The workspace is
        shared per B: runs that share it must be ordered on one stream."""
        B = labels.shape[0]
        if labels.shape[1:] != (self.H, self.W):
            raise ValueError(f"labels {tuple(labels.shape)} != (B, {self.H}, {self.W})")
        ws, rec = self._buffers(B)
        if out is not None:
            if (out.shape != rec.shape or out.dtype != rec.dtype or not out.is_contiguous()
                    or out.device != rec.device):
                raise ValueError("DevicePostprocess.run: out must be a contiguous [B, 1 + 5K] fp32 buffer")
            rec = out
        hip_ops.postprocess(labels, self.palette, ws, rec, B=B, H=self.H, W=self.W, crop_h=crop_h,
                            crop_w=crop_w, min_area=min_area, K=self.K, bins=self.bins, thr=self.thr,
                            accum=self.accum_for(B))
        return rec

    def fetch(self, rec: torch.Tensor, frame_ids: Sequence[int], ts: Sequence[float],
              streams: Sequence[int], W: int, H: int) -> np.ndarray:
        from ..parallel.dp import unpack_records
        B = rec.shape[0]
        h = self._host.get(B)
        if h is None:
            h = self._host[B] = torch.empty(rec.shape, dtype=torch.float32, pin_memory=True)
        h.copy_(rec, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return unpack_records(h.numpy(), self.K, frame_ids, ts, streams)
