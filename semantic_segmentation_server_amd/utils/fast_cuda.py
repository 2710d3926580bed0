"""Per-step stream switches and current-stream lookups without torch's per-call device
resolution.

``torch.cuda.stream(s)`` and ``torch.cuda.current_stream(None | torch.device)`` resolve the
device on every call (``_get_device_index`` -> ``is_available`` -> environment lookups): a
cProfile of the batch-1 step (scripts/profile_host.py, 2,000 steps) spent ~47 us of each
step in ``current_stream`` and ~36 us in the stream context managers, with the host on the
step's critical path (bench.py host_ms_per_step: busy ~0.10 of a ~0.17 ms step). Here the
device index is known (the pipeline's own device), so the switch is two C calls.
"""
from __future__ import annotations

import torch


class StreamSwitch:
    """``with StreamSwitch(s):`` == ``with torch.cuda.stream(s):`` for a stream on the
    current device (the pipeline's; switching devices is not supported here)."""

    __slots__ = ("_sid", "_idx", "_dt", "_prev")

    def __init__(self, stream: torch.cuda.Stream):
        self._sid, self._idx, self._dt = stream.stream_id, stream.device_index, stream.device_type
        self._prev = None

    def __enter__(self) -> "StreamSwitch":
        self._prev = torch._C._cuda_getCurrentStream(self._idx)
        torch._C._cuda_setStream(stream_id=self._sid, device_index=self._idx, device_type=self._dt)
        return self

    def __exit__(self, *exc) -> bool:
        p = self._prev
        torch._C._cuda_setStream(stream_id=p[0], device_index=p[1], device_type=p[2])
        return False


def current_stream(index: int) -> torch.cuda.Stream:
    """``torch.cuda.current_stream(index)`` for a known device index."""
    d = torch._C._cuda_getCurrentStream(index)
    return torch.cuda.Stream(stream_id=d[0], device_index=d[1], device_type=d[2])


def current_raw_stream() -> int:
    """The current stream's raw HIP handle on the current device (kernel launches)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())
