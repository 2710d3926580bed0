"""Pinned host -> device copy bandwidth at the bench's per-step ingest size
(32 x 480 x 640 x 3 B = 29.5 MB): one copy, and the same bytes split over
N concurrent copies on N streams (several SDMA engines)."""
import sys
import time

import torch


def run(nsplit, host, dev_buf, reps=20):
    streams = [torch.cuda.Stream() for _ in range(nsplit)]
    hs, ds = host.chunk(nsplit), dev_buf.chunk(nsplit)
    for _ in range(3):
        for s, h, d in zip(streams, hs, ds):
            with torch.cuda.stream(s):
                d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for s, h, d in zip(streams, hs, ds):
            with torch.cuda.stream(s):
                d.copy_(h, non_blocking=True)
        for s in streams:
            s.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return dt


def main():
    n = 32 * 480 * 640 * 3
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    host.random_(0, 255)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    for k in (1, 2, 4, 8):
        dt = run(k, host, dev)
        print(f"split {k}: {dt * 1e6:8.1f} us  {n / dt / 1e9:6.1f} GB/s", flush=True)


if __name__ == "__main__":
    sys.exit(main())
