"""Control plane in one process: coordinator + 2 client agents over localhost gRPC,
reference ("grpc") aggregation on CPU (BASELINE.json config 1: 2-layer MLP,
synthetic MNIST, 2 clients + 1 server)."""
import threading

import grpc
import pytest
import torch

from fedmi import ckpt as ck
from fedmi.control.client_agent import ClientAgent, serve_client
from fedmi.control.coordinator import Coordinator, CoordinatorConfig, fedavg_state_dicts
from fedmi.wire import proto as P

from helpers import free_port, small_trainer


@pytest.fixture()
def two_clients(tmp_path):
    agents, servers, addrs = [], [], []
    for i in range(2):
        addr = f"127.0.0.1:{free_port()}"
        ag = ClientAgent(small_trainer("mlp", seed=i), addr, root=tmp_path / f"c{i}", agg="grpc", verbose=False)
        srv, _ = serve_client(ag, addr)
        agents.append(ag)
        servers.append(srv)
        addrs.append(addr)
    yield agents, addrs
    for s in servers:
        s.stop(None)


def test_fedavg_state_dicts_semantics():
    a = {"w": torch.tensor([1.0, 3.0]), "n": torch.tensor(3)}
    b = {"w": torch.tensor([3.0, 5.0]), "n": torch.tensor(4)}
    out = fedavg_state_dicts([a, b])
    assert torch.equal(out["w"], torch.tensor([2.0, 4.0]))
    assert out["n"].dtype == torch.int64 and int(out["n"]) == 3     # float mean 3.5 truncated like the reference


def test_grpc_rounds_average_and_persist(tmp_path, two_clients):
    agents, addrs = two_clients
    cfg = CoordinatorConfig(clients=addrs, rounds=2, agg="grpc", root=str(tmp_path / "srv"), heartbeat_s=0.2,
                            train_timeout_s=60, rpc_timeout_s=10)
    coord = Coordinator(cfg)
    coord.run()
    coord.close()
    mount = tmp_path / "srv" / "Primary"
    assert coord.round == 2
    g = ck.load(mount / "optimizedModel.pth")
    assert g["epoch"] == 2 and set(g["net"]) == set(agents[0].trainer.state_dict())
    # after SendModel every client holds exactly the averaged model
    for ag in agents:
        for k, v in ag.trainer.state_dict().items():
            assert torch.allclose(v.cpu(), g["net"][k])
    # the average is the mean of this round's uploaded checkpoints
    t0, t1 = ck.load(mount / "test_0.pth")["net"], ck.load(mount / "test_1.pth")["net"]
    for k in g["net"]:
        assert torch.allclose(g["net"][k], (t0[k] + t1[k]) / 2, atol=1e-6)
    # client checkpoint files exist in the reference layout
    for i, a in enumerate(addrs):
        assert (tmp_path / f"c{i}" / "checkpoint" / f"{a}.pth").exists()


def test_dead_client_excluded_and_rejoins(tmp_path):
    addrs, agents, servers = [], [], []
    for i in range(2):
        addr = f"127.0.0.1:{free_port()}"
        ag = ClientAgent(small_trainer("mlp", seed=0), addr, root=tmp_path / f"c{i}", agg="grpc", verbose=False)
        addrs.append(addr)
        agents.append(ag)
        servers.append(serve_client(ag, addr)[0])
    cfg = CoordinatorConfig(clients=addrs, rounds=10, agg="grpc", root=str(tmp_path / "srv"), heartbeat_s=0.1,
                            train_timeout_s=30, rpc_timeout_s=2)
    coord = Coordinator(cfg)
    coord.start_tracker()
    assert coord.run_round()
    servers[1].stop(None)                       # client 1 dies
    coord.run_round()                           # failure detected, client 1 marked inactive
    assert coord.client_status()[addrs[1]] is False
    assert coord.run_round()                    # world = 1 now (quirk A5 fixed)
    r_before = coord.round
    servers[1] = serve_client(agents[1], addrs[1])[0]   # client 1 comes back
    ev = threading.Event()
    for _ in range(100):
        if coord.client_status()[addrs[1]]:
            break
        ev.wait(0.05)
    assert coord.client_status()[addrs[1]] is True
    # resynced with the latest global model on rejoin
    g = ck.from_bytes(coord.latest_model)["net"]
    for k, v in agents[1].trainer.state_dict().items():
        assert torch.allclose(v.cpu(), g[k])
    assert coord.run_round() and coord.round == r_before + 1
    coord.close()
    for s in servers:
        s.stop(None)


def test_stale_term_is_fenced(tmp_path, two_clients):
    agents, addrs = two_clients
    stub = P.TrainerStub(P.make_channel(addrs[0]))
    stub.StartTrain(P.TrainRequest(rank=0, world=1), timeout=30, metadata=[("x-fedmi-term", "200")])
    with pytest.raises(grpc.RpcError) as ei:
        stub.StartTrain(P.TrainRequest(rank=0, world=1), timeout=30, metadata=[("x-fedmi-term", "100")])
    assert ei.value.code() == grpc.StatusCode.FAILED_PRECONDITION
    with pytest.raises(grpc.RpcError) as ei:
        stub.StartTrain(P.TrainRequest(rank=2, world=2), timeout=30)
    assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_coordinator_resumes_round_from_checkpoint(tmp_path, two_clients):
    agents, addrs = two_clients
    root = str(tmp_path / "srv")
    c1 = Coordinator(CoordinatorConfig(clients=addrs, rounds=1, agg="grpc", root=root))
    c1.run()
    c1.close()
    c2 = Coordinator(CoordinatorConfig(clients=addrs, rounds=2, agg="grpc", root=root))
    assert c2.round == 1                        # quirk A8 fixed: the round survives a restart
    c2.run()
    c2.close()
    assert ck.load(tmp_path / "srv" / "Primary" / "optimizedModel.pth")["epoch"] == 2
