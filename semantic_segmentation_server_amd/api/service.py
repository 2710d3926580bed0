"""gRPC servicers, registration helpers and client stubs.

v1 ``sem_seg_server.SemanticSegmentation`` mirrors the reference servicer
(``sem_seg_server.py:216-234``) and its generated registration/stub code
(``sem_seg_server_pb2_grpc.py:8-63``): two unary-unary methods with ``Empty``
requests, ``GetSegmentedObjects`` pops exactly ``num_detections`` records
newest-first and pads with default ``SegmentedObject()`` messages, and
``GetCameraResolution`` returns the resolution probed once at startup. The RPC
never waits on inference.

v2 ``sem_seg_server.v2.SemanticSegmentationV2`` is new: per-stream reads with
frame ids/timestamps, stream listing, stats and health.
"""
from __future__ import annotations

import json
import time
from concurrent import futures
from typing import Callable, Dict, Optional, Tuple

import grpc

from . import proto as P
from ..labels import label_name
from ..runtime.results import ResultHub


def _obj(rec, labels) -> "P.SegmentedObject":
    return P.SegmentedObject(
        label=label_name(labels, int(rec["label"])),
        score=float(rec["score"]),
        area=float(rec["area"]),
        centroid=P.Centroid(cx=float(rec["cx"]), cy=float(rec["cy"])),
    )


class SemanticSegmentationServicer:
    """v1 service (reference-compatible)."""

    def __init__(self, hub: ResultHub, labels: Dict[int, str], num_detections: int = 3,
                 camera_res: Tuple[int, int] = (0, 0), stream: int = 0, metrics=None):
        self.hub = hub
        self.labels = labels
        self.num_detections = int(num_detections)
        self.camera_res = camera_res
        self.stream = stream
        self.metrics = metrics

    def GetCameraResolution(self, request, context):
        return P.CameraResolution(width=int(self.camera_res[0]), height=int(self.camera_res[1]))

    def GetSegmentedObjects(self, request, context):
        t0 = time.perf_counter()
        recs = self.hub.buffer(self.stream).pop(self.num_detections)
        data = [_obj(r, self.labels) for r in recs]
        data.extend(P.SegmentedObject() for _ in range(self.num_detections - len(data)))
        out = P.SegmentedObjectData(data=data)
        if self.metrics is not None:
            self.metrics.observe("rpc_get_segmented_objects_ms", (time.perf_counter() - t0) * 1e3)
        return out


MAX_V2_OBJECTS = 4096  # per-request cap of GetStreamSegmentedObjects (padding included)


class SemanticSegmentationV2Servicer:
    """v2 extension service. Client input is bounded: ``max_objects`` is clamped to
    [0, min(buffer capacity, MAX_V2_OBJECTS)] (a huge padded request would otherwise
    build billions of messages on the node's only RPC host) and an unknown
    ``stream_id`` is NOT_FOUND instead of creating a buffer."""

    def __init__(self, hub: ResultHub, labels: Dict[int, str], num_detections: int = 3,
                 streams: Optional[list] = None, metrics=None,
                 health_fn: Optional[Callable[[], Tuple[bool, int, int, str]]] = None):
        self.hub = hub
        self.labels = labels
        self.num_detections = int(num_detections)
        self.streams = streams or []
        self.metrics = metrics
        self.health_fn = health_fn

    def GetStreamSegmentedObjects(self, request, context):
        buf = self.hub.get(int(request.stream_id))
        if buf is None:
            context.set_code(grpc.StatusCode.NOT_FOUND)
            context.set_details(f"unknown stream_id {request.stream_id}")
            return P.StreamSegmentedObjects()
        cap = min(MAX_V2_OBJECTS, buf.maxlen or MAX_V2_OBJECTS)
        n = max(0, min(int(request.max_objects or self.num_detections), cap))
        recs = buf.pop(n)
        data = [P.TaggedObject(object=_obj(r, self.labels), frame_id=int(r["frame"]),
                               timestamp=float(r["ts"]), stream_id=int(r["stream"]))
                for r in recs]
        if request.pad:
            data.extend(P.TaggedObject(stream_id=request.stream_id) for _ in range(n - len(data)))
        return P.StreamSegmentedObjects(data=data)

    def ListStreams(self, request, context):
        return P.StreamList(streams=[P.StreamInfo(**s) for s in self.streams])

    def GetStats(self, request, context):
        snap = self.metrics.snapshot() if self.metrics is not None else {}
        fl = snap.get("frame_ms", {})
        return P.Stats(
            frames=int(snap.get("frames", 0)), fps=float(snap.get("fps", 0.0)),
            p50_frame_ms=float(fl.get("p50", 0.0)), p99_frame_ms=float(fl.get("p99", 0.0)),
            objects=int(snap.get("objects", 0)), buffer_depth=self.hub.depth,
            buffer_drops=self.hub.drops, json=json.dumps(snap, default=float))

    def Health(self, request, context):
        if self.health_fn is None:
            return P.HealthStatus(serving=True, ranks_alive=1, world_size=1, detail="ok")
        ok, alive, world, detail = self.health_fn()
        return P.HealthStatus(serving=ok, ranks_alive=alive, world_size=world, detail=detail)


def _handlers(servicer, methods: Dict[str, tuple]) -> Dict[str, grpc.RpcMethodHandler]:
    return {
        name: grpc.unary_unary_rpc_method_handler(
            getattr(servicer, name),
            request_deserializer=req.FromString,
            response_serializer=resp.SerializeToString)
        for name, (req, resp) in methods.items()
    }


def add_v1_servicer(servicer, server) -> None:
    server.add_generic_rpc_handlers(
        (grpc.method_handlers_generic_handler(P.V1_SERVICE, _handlers(servicer, P.V1_METHODS)),))


def add_v2_servicer(servicer, server) -> None:
    server.add_generic_rpc_handlers(
        (grpc.method_handlers_generic_handler(P.V2_SERVICE, _handlers(servicer, P.V2_METHODS)),))


class HealthServicer:
    """grpc.health.v1.Health. ``status_fn(service) -> bool | None`` (None = unknown
    service); "" and the two segmentation services are known. Watch streams the
    status whenever it changes (polled every ``watch_period`` s) until cancelled."""

    KNOWN = ("", P.V1_SERVICE, P.V2_SERVICE)

    def __init__(self, status_fn: Optional[Callable[[str], Optional[bool]]] = None,
                 watch_period: float = 0.5):
        self.status_fn = status_fn or (lambda service: True)
        self.watch_period = watch_period

    def _status(self, service: str) -> int:
        R = P.HealthCheckResponse
        if service not in self.KNOWN:
            return R.SERVICE_UNKNOWN
        ok = self.status_fn(service)
        return R.UNKNOWN if ok is None else (R.SERVING if ok else R.NOT_SERVING)

    def Check(self, request, context):
        st = self._status(request.service)
        if st == P.HealthCheckResponse.SERVICE_UNKNOWN:
            context.set_code(grpc.StatusCode.NOT_FOUND)
            context.set_details(f"unknown service {request.service!r}")
        return P.HealthCheckResponse(status=st)

    def Watch(self, request, context):
        last = None
        while context.is_active():
            st = self._status(request.service)
            if st != last:
                yield P.HealthCheckResponse(status=st)
                last = st
            time.sleep(self.watch_period)


def add_health_servicer(servicer: HealthServicer, server) -> None:
    handlers = {
        "Check": grpc.unary_unary_rpc_method_handler(
            servicer.Check, request_deserializer=P.HealthCheckRequest.FromString,
            response_serializer=P.HealthCheckResponse.SerializeToString),
        "Watch": grpc.unary_stream_rpc_method_handler(
            servicer.Watch, request_deserializer=P.HealthCheckRequest.FromString,
            response_serializer=P.HealthCheckResponse.SerializeToString),
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(P.HEALTH_SERVICE, handlers),))


class HealthStub:
    def __init__(self, channel):
        self.Check = channel.unary_unary(
            f"/{P.HEALTH_SERVICE}/Check", request_serializer=P.HealthCheckRequest.SerializeToString,
            response_deserializer=P.HealthCheckResponse.FromString)
        self.Watch = channel.unary_stream(
            f"/{P.HEALTH_SERVICE}/Watch", request_serializer=P.HealthCheckRequest.SerializeToString,
            response_deserializer=P.HealthCheckResponse.FromString)


class _Stub:
    def __init__(self, channel, service: str, methods: Dict[str, tuple]):
        for name, (req, resp) in methods.items():
            setattr(self, name, channel.unary_unary(
                f"/{service}/{name}",
                request_serializer=req.SerializeToString,
                response_deserializer=resp.FromString))


class SemanticSegmentationStub(_Stub):
    def __init__(self, channel):
        super().__init__(channel, P.V1_SERVICE, P.V1_METHODS)


class SemanticSegmentationV2Stub(_Stub):
    def __init__(self, channel):
        super().__init__(channel, P.V2_SERVICE, P.V2_METHODS)


def make_server(max_workers: int = 10, port: int = 50051, host: str = "[::]"):
    """grpc.server on its own thread pool (the reference shares one 10-thread pool
    between the producer and the RPC handlers, ``sem_seg_server.py:272-278``)."""
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers),
                         options=[("grpc.so_reuseport", 0)])
    bound = server.add_insecure_port(f"{host}:{port}")
    return server, bound
