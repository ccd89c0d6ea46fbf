"""End-to-end system on the MI355X: the reference's process layout (coordinator +
client processes speaking federated.proto over gRPC) with the native LeNet HIP
engine on the GPU.  Both clients share the box's one GPU; their FedAvg runs on
the GPU through the hipIpc peer kernels (csrc/comm/peer_comm.hip) -- RCCL
refuses two ranks on one GPU -- the transport a multi-GPU node uses over xGMI."""
import time

import pytest
import torch

from fedmi import ckpt as ck
from fedmi.control.coordinator import Coordinator, CoordinatorConfig

from helpers import free_port, read_jsonl, spawn_client, stop_proc, wait_heartbeat

pytestmark = pytest.mark.gpu


def _clients(tmp_path, n, extra=(), transport="peer"):
    addrs = [f"127.0.0.1:{free_port()}" for _ in range(n)]
    procs = [spawn_client(a, tmp_path, "--agg", "collective", "--model", "lenet", "--n-train", "2560",
                          "--n-test", "1000", "--transport", transport, "--metrics", str(tmp_path / f"client{i}.jsonl"),
                          *extra, log_path=tmp_path / f"client{i}.log", device="cuda:0")
             for i, a in enumerate(addrs)]
    for a in addrs:
        wait_heartbeat(a, timeout=100)
    return addrs, procs


@pytest.mark.parametrize("compress,transport", [(None, "peer"), ("Y", "peer"), ("topk", "peer"), (None, "auto")],
                         ids=["dense", "c-Y-int8", "topk", "dense-auto"])
def test_grpc_coordinator_drives_gpu_clients(tmp_path, compress, transport):
    extra = {None: (), "Y": ("-c", "Y"), "topk": ("-c", "Y", "--compress", "topk")}[compress]
    addrs, procs = _clients(tmp_path, 2, extra, transport=transport)
    try:
        cfg = CoordinatorConfig(clients=addrs, rounds=3, agg="collective", root=str(tmp_path / "srv"),
                                gzip=compress is not None, train_timeout_s=90, rpc_timeout_s=20, heartbeat_s=0.5)
        coord = Coordinator(cfg)
        coord.run()
        coord.close()
        assert coord.round == 3
        g = ck.load(tmp_path / "srv" / "Primary" / "optimizedModel.pth")
        assert g["epoch"] == 3
        assert list(g["net"]) == ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "fc1.weight",
                                  "fc1.bias", "fc2.weight", "fc2.bias", "fc3.weight", "fc3.bias"]
        assert all(torch.isfinite(v).all() for v in g["net"].values())
        for a in addrs:
            t0 = time.time()          # client checkpoints are written by a background writer
            while (ck.read_epoch(tmp_path / "checkpoint" / f"{a}.pth") or 0) < 3 and time.time() - t0 < 30:
                time.sleep(0.05)
            c = ck.load(tmp_path / "checkpoint" / f"{a}.pth")
            assert c["epoch"] == 3
            for k in g["net"]:
                assert torch.equal(c["net"][k], g["net"][k]), k     # rank-ordered peer sums: bit-identical
        if transport == "auto":
            # product path verify-and-select: two clients on one GPU cannot run RCCL, so the
            # peer kernel is verified against gloo at the first generation and kept
            for i in range(2):
                sel = [r["transport_select"] for r in read_jsonl(tmp_path / f"client{i}.jsonl")
                       if "transport_select" in r]
                assert sel and sel[0]["verified_against"] == "gloo" and sel[0]["chosen"] in ("oneshot", "twoshot")
    finally:
        for p in procs:
            stop_proc(p)
