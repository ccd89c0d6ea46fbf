"""A fedmi-speaking fake client process for control-plane tests (no training, no GPU):
``python tests/fake_client.py <port-file>`` serves federated.Trainer on an ephemeral port, writes the port to
<port-file> and honours round leases / fetches like fedmi.control.client_agent (see tests/test_lease.py)."""
import json
import sys
import threading
import time
from collections import OrderedDict
from pathlib import Path

import grpc
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from fedmi import ckpt as ck  # noqa: E402
from fedmi.control.client_agent import META_FETCH, META_HAVE, META_LEASE, META_ROUND, metadata_dict  # noqa: E402
from fedmi.wire import proto as P  # noqa: E402


def model_bytes(epoch: int, value: float) -> bytes:
    sd = OrderedDict([("w", torch.full((4,), float(value)))])
    return ck.to_bytes(ck.make_checkpoint(sd, acc=1, epoch=epoch))


class FakeClient(P.TrainerServicer):
    """'Trains' instantly: honours leases, reports per-round stats, serves the fetch path.  ``abort_at``:
    (round, committed) -> the lease fails at that round with ABORTED after committing ``committed``."""

    def __init__(self, work_s: float = 0.0):
        self.calls = 0
        self.rounds = 0
        self.ready = None            # (epoch, None): serialised on demand, like the writer's ready buffer
        self.installed = []          # epochs installed by SendModel (rollbacks / resyncs)
        self.abort_at = None
        self.lost_after_lease = False    # finish every round of the call, then fail UNAVAILABLE (died before replying)
        self.work_s = work_s
        self.lock = threading.Lock()

    def StartTrain(self, request, context):
        meta = metadata_dict(context)
        rnd = int(meta.get(META_ROUND, "1"))
        lease = int(meta.get(META_LEASE, "1"))
        with self.lock:
            self.calls += 1
        stats = []
        for r in range(rnd, rnd + lease):
            if self.abort_at is not None and r == self.abort_at[0]:
                committed = self.abort_at[1]
                self.ready = (committed, None)
                context.set_trailing_metadata((("x-fedmi-client-round", str(committed)),
                                               ("x-fedmi-ckpt-epoch", "-1")))
                context.abort(grpc.StatusCode.ABORTED, "peer collective timed out (a client was lost)")
            if self.work_s:
                time.sleep(self.work_s)
            self.rounds = r
            stats.append((r, 1.0 / r, 10.0 + r, time.time()))
        self.ready = (self.rounds, None)
        if self.lost_after_lease:
            context.abort(grpc.StatusCode.UNAVAILABLE, "Socket closed")
        context.set_trailing_metadata((("x-fedmi-client-round", str(self.rounds)),
                                       ("x-fedmi-ckpt-epoch", "-1"),
                                       ("x-fedmi-lease-stats", json.dumps(stats))))
        return P.TrainReply(message="")

    def SendModel(self, request, context):
        meta = metadata_dict(context)
        if meta.get(META_FETCH) == "1":
            have = int(meta.get(META_HAVE, "-1"))
            ready = self.ready
            epoch = ready[0] if ready else -1
            context.set_trailing_metadata((("x-fedmi-ckpt-epoch", str(epoch)),))
            return P.SendModelReply(reply=ck.to_b64(model_bytes(epoch, epoch)) if ready and epoch > have else "")
        self.installed.append(ck.from_bytes(ck.from_b64(request.model))["epoch"])
        self.ready = (self.installed[-1], None)
        return P.SendModelReply(reply="success")

    def HeartBeat(self, request, context):
        return P.HeartBeatResponse(status=1)


def serve(fake: FakeClient, workers: int = 4):
    srv = P.make_server(max_workers=workers)
    P.add_TrainerServicer_to_server(fake, srv)
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    return srv, port


if __name__ == "__main__":
    srv, port = serve(FakeClient())
    tmp = Path(sys.argv[1] + ".tmp")
    tmp.write_text(str(port))
    tmp.rename(sys.argv[1])
    srv.wait_for_termination()
