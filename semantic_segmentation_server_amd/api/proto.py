"""Protobuf message classes for the segmentation API, built without protoc.

The reference ships protoc-generated modules (``sem_seg_server_pb2.py``,
``sem_seg_server_pb2_grpc.py``) that only import under protobuf 3.x; protobuf in
this image is 7.x and there is no ``grpc_tools``. We therefore describe the two
files (``sem_seg_server.proto`` and the v2 extension) with ``descriptor_pb2``,
register them in a private ``DescriptorPool`` and materialise message classes with
``message_factory.GetMessageClass``. The resulting v1 wire format is identical to
the reference's (field numbers/types of ``sem_seg_server.proto:14-50``), which
``tests/test_api.py`` checks against hand-encoded bytes.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto

PACKAGE = "sem_seg_server"
V1_SERVICE = "sem_seg_server.SemanticSegmentation"
V2_PACKAGE = "sem_seg_server.v2"
V2_SERVICE = "sem_seg_server.v2.SemanticSegmentationV2"


def _field(msg, name, number, ftype, label=F.LABEL_OPTIONAL, type_name=None):
    f = msg.field.add()
    f.name = name
    f.number = number
    f.type = ftype
    f.label = label
    if type_name:
        f.type_name = type_name
    # proto3 JSON name convention
    parts = name.split("_")
    f.json_name = parts[0] + "".join(p.title() for p in parts[1:])
    return f


def _method(svc, name, inp, out):
    m = svc.method.add()
    m.name = name
    m.input_type = inp
    m.output_type = out
    return m


def v1_file_descriptor() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "sem_seg_server.proto"
    fd.package = PACKAGE
    fd.syntax = "proto3"

    so = fd.message_type.add()
    so.name = "SegmentedObject"
    cen = so.nested_type.add()
    cen.name = "Centroid"
    _field(cen, "cx", 1, F.TYPE_FLOAT)
    _field(cen, "cy", 2, F.TYPE_FLOAT)
    _field(so, "label", 1, F.TYPE_STRING)
    _field(so, "score", 2, F.TYPE_FLOAT)
    _field(so, "area", 3, F.TYPE_FLOAT)
    _field(so, "centroid", 4, F.TYPE_MESSAGE,
           type_name=".sem_seg_server.SegmentedObject.Centroid")

    sod = fd.message_type.add()
    sod.name = "SegmentedObjectData"
    _field(sod, "data", 1, F.TYPE_MESSAGE, F.LABEL_REPEATED, ".sem_seg_server.SegmentedObject")

    cr = fd.message_type.add()
    cr.name = "CameraResolution"
    _field(cr, "width", 1, F.TYPE_INT32)
    _field(cr, "height", 2, F.TYPE_INT32)

    em = fd.message_type.add()
    em.name = "Empty"

    svc = fd.service.add()
    svc.name = "SemanticSegmentation"
    _method(svc, "GetSegmentedObjects", ".sem_seg_server.Empty", ".sem_seg_server.SegmentedObjectData")
    _method(svc, "GetCameraResolution", ".sem_seg_server.Empty", ".sem_seg_server.CameraResolution")
    return fd


def v2_file_descriptor() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "sem_seg_server_v2.proto"
    fd.package = V2_PACKAGE
    fd.syntax = "proto3"
    fd.dependency.append("sem_seg_server.proto")
    P = "." + V2_PACKAGE + "."

    m = fd.message_type.add(); m.name = "StreamRequest"
    _field(m, "stream_id", 1, F.TYPE_INT32)
    _field(m, "max_objects", 2, F.TYPE_INT32)
    _field(m, "pad", 3, F.TYPE_BOOL)

    m = fd.message_type.add(); m.name = "TaggedObject"
    _field(m, "object", 1, F.TYPE_MESSAGE, type_name=".sem_seg_server.SegmentedObject")
    _field(m, "frame_id", 2, F.TYPE_INT64)
    _field(m, "timestamp", 3, F.TYPE_DOUBLE)
    _field(m, "stream_id", 4, F.TYPE_INT32)

    m = fd.message_type.add(); m.name = "StreamSegmentedObjects"
    _field(m, "data", 1, F.TYPE_MESSAGE, F.LABEL_REPEATED, P + "TaggedObject")

    m = fd.message_type.add(); m.name = "StreamInfo"
    _field(m, "stream_id", 1, F.TYPE_INT32)
    _field(m, "width", 2, F.TYPE_INT32)
    _field(m, "height", 3, F.TYPE_INT32)
    _field(m, "rank", 4, F.TYPE_INT32)
    _field(m, "source", 5, F.TYPE_STRING)

    m = fd.message_type.add(); m.name = "StreamList"
    _field(m, "streams", 1, F.TYPE_MESSAGE, F.LABEL_REPEATED, P + "StreamInfo")

    m = fd.message_type.add(); m.name = "Stats"
    _field(m, "frames", 1, F.TYPE_INT64)
    _field(m, "fps", 2, F.TYPE_DOUBLE)
    _field(m, "p50_frame_ms", 3, F.TYPE_DOUBLE)
    _field(m, "p99_frame_ms", 4, F.TYPE_DOUBLE)
    _field(m, "objects", 5, F.TYPE_INT64)
    _field(m, "buffer_depth", 6, F.TYPE_INT64)
    _field(m, "buffer_drops", 7, F.TYPE_INT64)
    _field(m, "json", 8, F.TYPE_STRING)

    m = fd.message_type.add(); m.name = "HealthStatus"
    _field(m, "serving", 1, F.TYPE_BOOL)
    _field(m, "ranks_alive", 2, F.TYPE_INT32)
    _field(m, "world_size", 3, F.TYPE_INT32)
    _field(m, "detail", 4, F.TYPE_STRING)

    svc = fd.service.add()
    svc.name = "SemanticSegmentationV2"
    E = ".sem_seg_server.Empty"
    _method(svc, "GetStreamSegmentedObjects", P + "StreamRequest", P + "StreamSegmentedObjects")
    _method(svc, "ListStreams", E, P + "StreamList")
    _method(svc, "GetStats", E, P + "Stats")
    _method(svc, "Health", E, P + "HealthStatus")
    return fd


HEALTH_SERVICE = "grpc.health.v1.Health"


def health_file_descriptor() -> descriptor_pb2.FileDescriptorProto:
    """The standard gRPC health-checking protocol (grpc/health/v1/health.proto),
    so stock probes (grpc_health_probe, load balancers, k8s) can query the server
    without grpcio-health-checking installed."""
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "grpc/health/v1/health.proto"
    fd.package = "grpc.health.v1"
    fd.syntax = "proto3"
    m = fd.message_type.add(); m.name = "HealthCheckRequest"
    _field(m, "service", 1, F.TYPE_STRING)
    m = fd.message_type.add(); m.name = "HealthCheckResponse"
    e = m.enum_type.add(); e.name = "ServingStatus"
    for i, n in enumerate(["UNKNOWN", "SERVING", "NOT_SERVING", "SERVICE_UNKNOWN"]):
        v = e.value.add(); v.name = n; v.number = i
    _field(m, "status", 1, F.TYPE_ENUM,
           type_name=".grpc.health.v1.HealthCheckResponse.ServingStatus")
    svc = fd.service.add(); svc.name = "Health"
    _method(svc, "Check", ".grpc.health.v1.HealthCheckRequest", ".grpc.health.v1.HealthCheckResponse")
    w = _method(svc, "Watch", ".grpc.health.v1.HealthCheckRequest", ".grpc.health.v1.HealthCheckResponse")
    w.server_streaming = True
    return fd


POOL = descriptor_pool.DescriptorPool()
_V1_FD = POOL.Add(v1_file_descriptor())
_V2_FD = POOL.Add(v2_file_descriptor())
_HEALTH_FD = POOL.Add(health_file_descriptor())


def _cls(full_name: str):
    return message_factory.GetMessageClass(POOL.FindMessageTypeByName(full_name))


# ---- v1 (reference-compatible) -------------------------------------------
SegmentedObject = _cls("sem_seg_server.SegmentedObject")
Centroid = SegmentedObject.Centroid
SegmentedObjectData = _cls("sem_seg_server.SegmentedObjectData")
CameraResolution = _cls("sem_seg_server.CameraResolution")
Empty = _cls("sem_seg_server.Empty")

# ---- v2 (extension) --------------------------------------------------------
StreamRequest = _cls("sem_seg_server.v2.StreamRequest")
TaggedObject = _cls("sem_seg_server.v2.TaggedObject")
StreamSegmentedObjects = _cls("sem_seg_server.v2.StreamSegmentedObjects")
StreamInfo = _cls("sem_seg_server.v2.StreamInfo")
StreamList = _cls("sem_seg_server.v2.StreamList")
Stats = _cls("sem_seg_server.v2.Stats")
HealthStatus = _cls("sem_seg_server.v2.HealthStatus")

# ---- grpc.health.v1 ---------------------------------------------------------
HealthCheckRequest = _cls("grpc.health.v1.HealthCheckRequest")
HealthCheckResponse = _cls("grpc.health.v1.HealthCheckResponse")

V1_METHODS = {
    "GetSegmentedObjects": (Empty, SegmentedObjectData),
    "GetCameraResolution": (Empty, CameraResolution),
}
V2_METHODS = {
    "GetStreamSegmentedObjects": (StreamRequest, StreamSegmentedObjects),
    "ListStreams": (Empty, StreamList),
    "GetStats": (Empty, Stats),
    "Health": (Empty, HealthStatus),
}


def file_descriptor_set_bytes() -> bytes:
    """Serialized FileDescriptorSet of both files (for reflection/debugging)."""
    s = descriptor_pb2.FileDescriptorSet()
    s.file.add().CopyFrom(v1_file_descriptor())
    s.file.add().CopyFrom(v2_file_descriptor())
    s.file.add().CopyFrom(health_file_descriptor())
    return s.SerializeToString()
