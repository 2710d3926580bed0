"""Single configuration dataclass + CLI.

Reference flags (``sem_seg_server.py:236-260``) are kept with the same names and
defaults: ``--model``, ``--labels``, ``--keep_aspect_ratio`` (default True — made a
real toggle via ``--no_keep_aspect_ratio``; the reference's ``store_true`` plus
``set_defaults(True)`` could never turn it off), ``--camera_idx`` (1),
``--num_detections`` (3), ``--min_area_ratio`` (0.05). The reference's hard-coded
port 50051 (``:281``) and pool size 10 (``:272``) become ``--port`` and
``--max_workers``. Everything else is new.
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field
from typing import List, Optional

from .labels import CITYSCAPES_LABELS, PASCAL_LABELS


@dataclass
class Config:
    # --- reference flags ---
    model: Optional[str] = None            # optional weights file (.pt state_dict / .safetensors)
    labels: str = PASCAL_LABELS
    keep_aspect_ratio: bool = True
    camera_idx: int = 1
    num_detections: int = 3
    min_area_ratio: float = 0.05
    # --- serving ---
    port: int = 50051
    host: str = "[::]"
    max_workers: int = 10
    buffer_max: Optional[int] = 4096       # None = unbounded (reference semantics)
    # --- sources ---
    source: str = "synthetic"              # synthetic | file | camera
    source_path: Optional[str] = None
    camera_width: int = 640
    camera_height: int = 480
    streams: int = 1                       # camera streams per rank
    fps_limit: Optional[float] = None
    # --- model ---
    arch: str = "mnv2"                     # mnv2 | resnet50
    num_classes: int = 21
    dataset: str = "pascal"                # palette for the mask stage
    width_mult: float = 1.0
    output_stride: int = 16
    aspp: str = "full"                     # full | mobile
    input_size: int = 513
    seed: int = 0
    # --- execution ---
    backend: str = "hip"                   # hip | torch
    dtype: str = "bf16"                    # bf16 | fp32 | int8
    device: str = "auto"                   # auto | cpu | cuda
    batch: int = 1                         # frames per rank per step
    graph: bool = True                     # hipGraph capture of the per-step device work
    contour_mode: str = "fast"             # fast (device CCL stats) | exact (host tracer)
    max_segments: int = 64                 # per-frame record capacity on device
    # --- distributed ---
    gpus: int = 1
    ingest: str = "local"                  # local (per-rank H2D) | scatter (rank-0 RCCL scatter)
    gather: str = "auto"                   # record gather to rank 0: auto (= host) | host
                                           # (pinned host + gloo) | rccl (RCCL over xGMI)
    # --- observability ---
    profile: bool = False
    metrics_dump: Optional[str] = None
    log_level: str = "INFO"
    inject_fault: Optional[str] = None     # "rank:step" fault injection for tests
    rank_timeout: float = 300.0            # process-group collective timeout (s)
    degrade: bool = True                   # rank 0 keeps serving alone when a peer rank is lost
    debug_dump: Optional[str] = None       # directory for annotated PNG frames (reference :196-205)
    debug_every: int = 0                   # dump every N-th frame (0 = off)
    debug_sync: bool = False               # HIP_LAUNCH_BLOCKING=1, eager launches
    supervise: bool = True                 # CLI: GPU work in supervised worker processes (one per GPU)

    @property
    def min_area(self) -> float:
        return self.min_area_ratio * self.input_size * self.input_size

    def replace(self, **kw) -> "Config":
        return dataclasses.replace(self, **kw)

    def resolve_dataset_defaults(self) -> "Config":
        if self.dataset == "cityscapes" and self.labels == PASCAL_LABELS:
            self.labels = CITYSCAPES_LABELS
        return self


def add_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    d = Config()
    # reference flags, same names/defaults
    p.add_argument("--model", default=d.model, help="optional weights file (torch state_dict or safetensors); random init if omitted")
    p.add_argument("--labels", default=d.labels, help="label file path")
    p.add_argument("--keep_aspect_ratio", dest="keep_aspect_ratio", action="store_true",
                   help="keep the image aspect ratio when resizing, padding bottom/right with zeros (default)")
    p.add_argument("--no_keep_aspect_ratio", dest="keep_aspect_ratio", action="store_false",
                   help="stretch frames to the model input instead of letterboxing")
    p.set_defaults(keep_aspect_ratio=True)
    p.add_argument("--camera_idx", type=int, default=d.camera_idx, help="index of the video source")
    p.add_argument("--num_detections", type=int, default=d.num_detections, help="number of detections to return")
    p.add_argument("--min_area_ratio", type=float, default=d.min_area_ratio, help="segment centroid min area ratio")
    # new
    p.add_argument("--port", type=int, default=d.port)
    p.add_argument("--host", default=d.host)
    p.add_argument("--max_workers", type=int, default=d.max_workers)
    p.add_argument("--buffer_max", type=int, default=d.buffer_max, help="result buffer bound; 0 = unbounded")
    p.add_argument("--source", choices=["synthetic", "file", "camera"], default=d.source)
    p.add_argument("--source_path", default=d.source_path)
    p.add_argument("--camera_width", type=int, default=d.camera_width)
    p.add_argument("--camera_height", type=int, default=d.camera_height)
    p.add_argument("--streams", type=int, default=d.streams)
    p.add_argument("--fps_limit", type=float, default=d.fps_limit)
    p.add_argument("--arch", choices=["mnv2", "resnet50"], default=d.arch)
    p.add_argument("--num_classes", type=int, default=d.num_classes)
    p.add_argument("--dataset", choices=["pascal", "cityscapes"], default=d.dataset)
    p.add_argument("--width_mult", type=float, default=d.width_mult)
    p.add_argument("--output_stride", type=int, default=d.output_stride)
    p.add_argument("--aspp", choices=["full", "mobile"], default=d.aspp)
    p.add_argument("--input_size", type=int, default=d.input_size)
    p.add_argument("--seed", type=int, default=d.seed)
    p.add_argument("--backend", choices=["hip", "torch"], default=d.backend)
    p.add_argument("--dtype", choices=["bf16", "fp32", "int8"], default=d.dtype)
    p.add_argument("--device", default=d.device)
    p.add_argument("--batch", type=int, default=d.batch)
    p.add_argument("--graph", dest="graph", action="store_true")
    p.add_argument("--no-graph", "--no_graph", dest="graph", action="store_false")
    p.set_defaults(graph=d.graph)
    p.add_argument("--contour_mode", choices=["fast", "exact"], default=d.contour_mode)
    p.add_argument("--max_segments", type=int, default=d.max_segments)
    p.add_argument("--gpus", type=int, default=d.gpus)
    p.add_argument("--ingest", choices=["local", "scatter"], default=d.ingest)
    p.add_argument("--gather", choices=["auto", "rccl", "host"], default=d.gather,
                   help="per-step record gather to rank 0: pinned host memory over gloo "
                        "(auto; no GPU time) or RCCL over xGMI (rccl)")
    p.add_argument("--profile", action="store_true")
    p.add_argument("--metrics_dump", default=d.metrics_dump)
    p.add_argument("--log_level", default=d.log_level)
    p.add_argument("--inject_fault", default=d.inject_fault)
    p.add_argument("--rank_timeout", type=float, default=d.rank_timeout)
    p.add_argument("--no_degrade", dest="degrade", action="store_false",
                   help="exit instead of serving from rank 0 alone when a peer rank is lost")
    p.add_argument("--debug_dump", default=d.debug_dump,
                   help="write annotated PNG frames here (contours, centroids, labels)")
    p.add_argument("--debug_every", type=int, default=d.debug_every)
    p.add_argument("--debug_sync", action="store_true",
                   help="synchronous kernel launches (HIP_LAUNCH_BLOCKING=1, no hipGraph) so a "
                        "faulting kernel is reported at its own launch")
    p.add_argument("--no_supervise", dest="supervise", action="store_false",
                   help="run the GPU pipeline in the serving process itself (no restart of a "
                        "faulted worker)")
    return p


def apply_debug_env(cfg: Config) -> Config:
    """--debug_sync: must run before anything initialises the HIP runtime (the
    variable is read once, at runtime init). hipGraph capture is turned off too:
    a graph replays its kernels as one submission, which would hide the culprit."""
    if cfg.debug_sync:
        os.environ["HIP_LAUNCH_BLOCKING"] = "1"
        cfg = dataclasses.replace(cfg, graph=False)
    return cfg


def from_args(args: argparse.Namespace) -> Config:
    kw = {f.name: getattr(args, f.name) for f in dataclasses.fields(Config) if hasattr(args, f.name)}
    if kw.get("buffer_max") == 0:
        kw["buffer_max"] = None
    return Config(**kw).resolve_dataset_defaults()


def parse(argv: Optional[List[str]] = None) -> Config:
    p = add_args(argparse.ArgumentParser(description="MI355X semantic segmentation server"))
    return from_args(p.parse_args(argv))
