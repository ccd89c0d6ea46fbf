"""Wire compatibility of the programmatic federated.proto with the reference.

The reference's generated module (/root/reference/src/federated_pb2*.py, public
source, read-only) is imported when present; its serialized descriptor and
message bytes must equal ours, and its stubs must talk to our servers.
"""
import base64
import re
import sys
from pathlib import Path

import grpc
import pytest

from fedmi.wire import proto as P

REF_SRC = Path("/root/reference/src")
ROOT = Path(__file__).resolve().parent.parent


def _ref_modules():
    if not (REF_SRC / "federated_pb2.py").exists():
        pytest.skip("reference sources not mounted")
    sys.path.insert(0, str(REF_SRC))
    try:
        import federated_pb2 as R  # noqa: N812
        import federated_pb2_grpc as RG  # noqa: N812
    finally:
        sys.path.remove(str(REF_SRC))
    return R, RG


def test_messages_and_fields_match_proto_file():
    text = (ROOT / "proto" / "federated.proto").read_text()
    for name, fields in P.MESSAGES.items():
        m = re.search(r"message\s+%s\s*\{([^}]*)\}" % name, text)
        assert m, name
        body = m.group(1)
        for fname, num, _ in fields:
            assert re.search(r"\b%s\s*=\s*%d\s*;" % (fname, num), body), (name, fname)
    for rpc, (req, resp) in P.METHODS.items():
        assert re.search(r"rpc\s+%s\s*\(\s*%s\s*\)\s*returns\s*\(\s*%s\s*\)" % (rpc, req, resp), text), rpc
    assert "package federated;" in text


def test_roundtrip_and_string_payload():
    r = P.TrainRequest(rank=3, world=8)
    assert P.TrainRequest.FromString(r.SerializeToString()) == r
    payload = base64.b64encode(b"\x00\x01ckpt").decode()
    rep = P.TrainReply(message=payload)
    assert P.TrainReply.FromString(rep.SerializeToString()).message == payload


def test_descriptor_and_bytes_identical_to_reference():
    R, _ = _ref_modules()
    ours = P.file_descriptor_proto()
    from google.protobuf import descriptor_pb2

    theirs = descriptor_pb2.FileDescriptorProto.FromString(R.DESCRIPTOR.serialized_pb)
    assert theirs.package == ours.package and theirs.syntax == ours.syntax
    assert [m.name for m in theirs.message_type] == [m.name for m in ours.message_type]
    for mt, mo in zip(theirs.message_type, ours.message_type):
        assert [(f.name, f.number, f.type, f.label) for f in mt.field] == \
               [(f.name, f.number, f.type, f.label) for f in mo.field]
    (st,), (so,) = theirs.service, ours.service
    assert [(m.name, m.input_type, m.output_type) for m in st.method] == \
           [(m.name, m.input_type, m.output_type) for m in so.method]
    samples = [("TrainRequest", dict(rank=1, world=2)), ("TrainReply", dict(message="abc")),
               ("SendModelRequest", dict(model="QUJD")), ("SendModelReply", dict(reply="success")),
               ("PingRequest", dict(req="1")), ("PingResponse", dict(value=1)),
               ("HeartBeatResponse", dict(status=1)), ("Request", {})]
    for name, kw in samples:
        assert getattr(R, name)(**kw).SerializeToString() == getattr(P, name)(**kw).SerializeToString()


class _Echo(P.TrainerServicer):
    def StartTrain(self, request, context):
        return P.TrainReply(message=f"{request.rank}/{request.world}")

    def HeartBeat(self, request, context):
        return P.HeartBeatResponse(status=1)


def test_reference_stub_talks_to_fedmi_server():
    R, RG = _ref_modules()
    server = P.make_server(max_workers=2)
    P.add_TrainerServicer_to_server(_Echo(), server)
    port = server.add_insecure_port("127.0.0.1:0")
    server.start()
    try:
        ch = grpc.insecure_channel(f"127.0.0.1:{port}")
        stub = RG.TrainerStub(ch)
        assert stub.StartTrain(R.TrainRequest(rank=1, world=4), timeout=5).message == "1/4"
        assert stub.HeartBeat(R.Request(), timeout=5).status == 1
        with pytest.raises(grpc.RpcError) as ei:
            stub.SendModel(R.SendModelRequest(model=""), timeout=5)
        assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
    finally:
        server.stop(None)


def test_fedmi_stub_talks_to_reference_servicer():
    R, RG = _ref_modules()

    class RefStyle(RG.TrainerServicer):
        def CheckIfPrimaryUp(self, request, context):
            return R.PingResponse(value=int(request.req) + 1)

    server = grpc.server(__import__("concurrent.futures").futures.ThreadPoolExecutor(2))
    RG.add_TrainerServicer_to_server(RefStyle(), server)
    port = server.add_insecure_port("127.0.0.1:0")
    server.start()
    try:
        stub = P.TrainerStub(P.make_channel(f"127.0.0.1:{port}", gzip=True))
        assert stub.CheckIfPrimaryUp(P.PingRequest(req="1"), timeout=5).value == 2
    finally:
        server.stop(None)
