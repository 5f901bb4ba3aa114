"""Protobuf message classes for ``node_service.proto`` built without protoc.

The reference ships protoc-generated modules pinned to protobuf 5.29 / grpcio
1.71 (``node_service_pb2.py:12-19``, ``node_service_pb2_grpc.py:8-25``).  The
image has no ``grpc_tools``; instead the ``FileDescriptorProto`` is assembled
here field by field from ``node_service.proto`` and turned into message classes
with the runtime's message factory, so the encoding is byte-identical with the
reference's generated code (pinned by ``tests/test_wire.py``).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool

try:  # protobuf >= 4.21
    from google.protobuf.message_factory import GetMessageClass as _get_class
except ImportError:  # pragma: no cover
    from google.protobuf import message_factory as _mf
    _get_class = lambda d: _mf.MessageFactory().GetPrototype(d)  # noqa: E731

PACKAGE = "node_service"
SERVICE = "NodeService"
SERVICE_FULL = f"{PACKAGE}.{SERVICE}"

_F = descriptor_pb2.FieldDescriptorProto


def _file_descriptor() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="node_service.proto", package=PACKAGE, syntax="proto3")

    def msg(name, *fields, oneofs=()):
        m = fd.message_type.add(name=name)
        for o in oneofs:
            m.oneof_decl.add(name=o)
        for f in fields:
            m.field.add(**f)
        return m

    def fld(name, num, typ, label=_F.LABEL_OPTIONAL, type_name=None, **kw):
        d = dict(name=name, number=num, type=typ, label=label, json_name=_json(name))
        if type_name:
            d["type_name"] = type_name
        d.update(kw)
        return d

    msg("MessageRequest", fld("sender_id", 1, _F.TYPE_STRING), fld("message_text", 2, _F.TYPE_STRING))
    msg("MessageReply", fld("confirmation_text", 1, _F.TYPE_STRING))
    msg("Empty")
    msg("HealthCheckResponse", fld("is_healthy", 1, _F.TYPE_BOOL))
    msg("Tensor", fld("tensor_data", 1, _F.TYPE_BYTES),
        fld("shape", 2, _F.TYPE_INT32, label=_F.LABEL_REPEATED),
        fld("dtype", 3, _F.TYPE_STRING))
    msg("TensorRequest", fld("request_id", 1, _F.TYPE_STRING),
        fld("tensor", 2, _F.TYPE_MESSAGE, type_name=f".{PACKAGE}.Tensor"))
    # proto3 `optional` = synthetic oneof `_result_tensor` + proto3_optional flag
    msg("TensorResponse", fld("status", 1, _F.TYPE_STRING),
        fld("result_tensor", 2, _F.TYPE_MESSAGE, type_name=f".{PACKAGE}.Tensor",
            oneof_index=0, proto3_optional=True),
        oneofs=("_result_tensor",))
    svc = fd.service.add(name=SERVICE)
    for name, i, o in (("SendMessage", "MessageRequest", "MessageReply"),
                       ("HealthCheck", "Empty", "HealthCheckResponse"),
                       ("SendTensor", "TensorRequest", "TensorResponse")):
        svc.method.add(name=name, input_type=f".{PACKAGE}.{i}", output_type=f".{PACKAGE}.{o}")
    return fd


def _json(name: str) -> str:
    head, *rest = name.split("_")
    return head + "".join(p.capitalize() for p in rest)


def _build():
    pool = descriptor_pool.DescriptorPool()
    fdesc = pool.Add(_file_descriptor())
    fdesc = pool.FindFileByName("node_service.proto")
    classes = {n: _get_class(fdesc.message_types_by_name[n]) for n in fdesc.message_types_by_name}
    return fdesc, classes


FILE_DESCRIPTOR, _CLASSES = _build()
MessageRequest = _CLASSES["MessageRequest"]
MessageReply = _CLASSES["MessageReply"]
Empty = _CLASSES["Empty"]
HealthCheckResponse = _CLASSES["HealthCheckResponse"]
Tensor = _CLASSES["Tensor"]
TensorRequest = _CLASSES["TensorRequest"]
TensorResponse = _CLASSES["TensorResponse"]

METHODS = {
    "SendMessage": (MessageRequest, MessageReply),
    "HealthCheck": (Empty, HealthCheckResponse),
    "SendTensor": (TensorRequest, TensorResponse),
}


def method_path(name: str) -> str:
    return f"/{SERVICE_FULL}/{name}"
