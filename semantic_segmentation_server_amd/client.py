"""Example client and RPC latency benchmark.

``run()`` mirrors the reference client (``sem_seg_client.py:11-40``): an insecure
channel to ``localhost:50051`` and an endless loop alternating
``GetCameraResolution`` and ``GetSegmentedObjects``, printing the responses; on an
``RpcError`` it prints details and code and exits with status 1. ``--count``
bounds the loop (the reference's is infinite with no sleep).

``rpc_latency()`` measures the p50/p99 of ``GetSegmentedObjects`` — the latency
half of the headline metric (BASELINE.json).
"""
from __future__ import annotations

import argparse
import sys
import time
from typing import Dict, List, Optional

import grpc
import numpy as np

from .api import proto as P
from .api.service import SemanticSegmentationStub, SemanticSegmentationV2Stub


def get_camera_resolution(stub):
    try:
        response = stub.GetCameraResolution(P.Empty())
        print("Camera resolution fetched.")
        return response
    except grpc.RpcError as err:
        print(err.details())
        print("{}, {}".format(err.code().name, err.code().value))
        sys.exit(1)


def get_detected_objects(stub):
    try:
        response = stub.GetSegmentedObjects(P.Empty())
        print("Detected object(s) fetched.")
        return response
    except grpc.RpcError as err:
        print(err.details())
        print("{}, {}".format(err.code().name, err.code().value))
        sys.exit(1)


def run(target: str = "localhost:50051", count: Optional[int] = None) -> None:
    with grpc.insecure_channel(target) as channel:
        stub = SemanticSegmentationStub(channel)
        i = 0
        while count is None or i < count:
            print(get_camera_resolution(stub))
            print(get_detected_objects(stub))
            i += 1


def rpc_latency(target: str, n: int = 2000, warmup: int = 200) -> Dict[str, float]:
    """Sequential GetSegmentedObjects round trips over one channel."""
    with grpc.insecure_channel(target) as channel:
        stub = SemanticSegmentationStub(channel)
        grpc.channel_ready_future(channel).result(timeout=30)
        for _ in range(warmup):
            stub.GetSegmentedObjects(P.Empty())
        lat: List[float] = []
        for _ in range(n):
            t0 = time.perf_counter()
            stub.GetSegmentedObjects(P.Empty())
            lat.append((time.perf_counter() - t0) * 1e3)
    a = np.asarray(lat)
    return {"p50_ms": float(np.percentile(a, 50)), "p99_ms": float(np.percentile(a, 99)),
            "mean_ms": float(a.mean()), "n": n}


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="sem_seg_server example client")
    p.add_argument("--target", default="localhost:50051")
    p.add_argument("--count", type=int, default=None)
    p.add_argument("--latency", action="store_true", help="measure GetSegmentedObjects latency")
    p.add_argument("--stats", action="store_true", help="print v2 GetStats")
    a = p.parse_args(argv)
    if a.latency:
        print(rpc_latency(a.target))
        return 0
    if a.stats:
        with grpc.insecure_channel(a.target) as ch:
            print(SemanticSegmentationV2Stub(ch).GetStats(P.Empty()))
        return 0
    run(a.target, a.count)
    return 0


if __name__ == "__main__":
    sys.exit(main())
