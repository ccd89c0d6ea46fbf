"""``federated.proto`` built programmatically + hand-written gRPC glue.

The runtime image has grpcio/protobuf but no protoc/grpc_tools, so instead of
checking in generated ``*_pb2.py`` files the file descriptor is assembled here
with ``descriptor_pb2`` (same package ``federated``, service ``Trainer``, 4
unary RPCs, 8 messages, identical field numbers/types as the reference's
``federated.proto:22-63``).  It is registered in a PRIVATE descriptor pool so
the reference's generated module can be imported in the same process (wire
compatibility tests) without a duplicate-file conflict.
"""
from __future__ import annotations

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "federated"
SERVICE = "Trainer"
FULL_SERVICE = f"{PACKAGE}.{SERVICE}"

_I32 = descriptor_pb2.FieldDescriptorProto.TYPE_INT32
_STR = descriptor_pb2.FieldDescriptorProto.TYPE_STRING

# message name -> [(field, number, type)]
MESSAGES = {
    "Request": [],
    "HeartBeatResponse": [("status", 1, _I32)],
    "TrainRequest": [("rank", 1, _I32), ("world", 2, _I32)],
    "TrainReply": [("message", 1, _STR)],
    "SendModelRequest": [("model", 1, _STR)],
    "SendModelReply": [("reply", 1, _STR)],
    "PingRequest": [("req", 1, _STR)],
    "PingResponse": [("value", 1, _I32)],
}

# rpc name -> (request, response)
METHODS = {
    "StartTrain": ("TrainRequest", "TrainReply"),
    "SendModel": ("SendModelRequest", "SendModelReply"),
    "HeartBeat": ("Request", "HeartBeatResponse"),
    "CheckIfPrimaryUp": ("PingRequest", "PingResponse"),
}


def file_descriptor_proto() -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto(name="federated.proto", package=PACKAGE, syntax="proto3")
    fdp.options.java_multiple_files = True
    fdp.options.java_package = "io.grpc.examples.federated"
    fdp.options.java_outer_classname = "FederatedProto"
    fdp.options.objc_class_prefix = "HLW"
    for name, fields in MESSAGES.items():
        m = fdp.message_type.add(name=name)
        for fname, num, ftype in fields:
            m.field.add(name=fname, number=num, type=ftype,
                        label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL, json_name=fname)
    svc = fdp.service.add(name=SERVICE)
    for rpc, (req, resp) in METHODS.items():
        svc.method.add(name=rpc, input_type=f".{PACKAGE}.{req}", output_type=f".{PACKAGE}.{resp}")
    return fdp


POOL = descriptor_pool.DescriptorPool()
FILE = POOL.Add(file_descriptor_proto())
_classes = {name: message_factory.GetMessageClass(POOL.FindMessageTypeByName(f"{PACKAGE}.{name}"))
            for name in MESSAGES}

Request = _classes["Request"]
HeartBeatResponse = _classes["HeartBeatResponse"]
TrainRequest = _classes["TrainRequest"]
TrainReply = _classes["TrainReply"]
SendModelRequest = _classes["SendModelRequest"]
SendModelReply = _classes["SendModelReply"]
PingRequest = _classes["PingRequest"]
PingResponse = _classes["PingResponse"]


def method_path(rpc: str) -> str:
    return f"/{FULL_SERVICE}/{rpc}"


class TrainerStub:
    """Client-side stub: one callable per RPC (same surface as a generated stub)."""

    def __init__(self, channel: grpc.Channel):
        for rpc, (req, resp) in METHODS.items():
            setattr(self, rpc, channel.unary_unary(
                method_path(rpc),
                request_serializer=_classes[req].SerializeToString,
                response_deserializer=_classes[resp].FromString))


class TrainerServicer:
    """Server-side base: unimplemented RPCs answer UNIMPLEMENTED."""

    def _unimplemented(self, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method not implemented!")
        raise NotImplementedError("Method not implemented!")

    def StartTrain(self, request, context):
        self._unimplemented(context)

    def SendModel(self, request, context):
        self._unimplemented(context)

    def HeartBeat(self, request, context):
        self._unimplemented(context)

    def CheckIfPrimaryUp(self, request, context):
        self._unimplemented(context)


def add_TrainerServicer_to_server(servicer: TrainerServicer, server: grpc.Server) -> None:
    handlers = {
        rpc: grpc.unary_unary_rpc_method_handler(
            getattr(servicer, rpc),
            request_deserializer=_classes[req].FromString,
            response_serializer=_classes[resp].SerializeToString)
        for rpc, (req, resp) in METHODS.items()
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(FULL_SERVICE, handlers),))


# ---- transport options shared by every channel/server (reference: 1 GiB limits) --------
MAX_MSG = 1024 * 1024 * 1024
CHANNEL_OPTIONS = [
    ("grpc.max_send_message_length", MAX_MSG),
    ("grpc.max_receive_message_length", MAX_MSG),
]


# A peer that is not up yet (a backup still importing, a restarting client) must not push the
# channel into gRPC's default exponential reconnect backoff (up to 120 s): liveness pings and
# rejoin probes would then miss the peer for minutes.  Reconnect at most every second.
RECONNECT_OPTIONS = [
    ("grpc.initial_reconnect_backoff_ms", 100),
    ("grpc.min_reconnect_backoff_ms", 100),
    ("grpc.max_reconnect_backoff_ms", 1000),
]


def make_channel(address: str, gzip: bool = False) -> grpc.Channel:
    comp = grpc.Compression.Gzip if gzip else None
    return grpc.insecure_channel(address, options=CHANNEL_OPTIONS + RECONNECT_OPTIONS, compression=comp)


def make_server(max_workers: int = 10, gzip: bool = False) -> grpc.Server:
    from concurrent import futures

    comp = grpc.Compression.Gzip if gzip else None
    return grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers), options=CHANNEL_OPTIONS,
                       compression=comp)
