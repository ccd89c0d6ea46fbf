"""Round leases (x-fedmi-lease): one StartTrain covers K consecutive rounds, so the control-plane round trip
is paid once per lease (reference cadence: one StartTrain fan-out per round,
src/server.py:120-153).

* in-process fake clients (real gRPC servers, no training): the coordinator's per-round overhead with a
  lease is a fraction of the per-round-RPC overhead and stays flat from 1 to 8 clients;
* an aborted lease whose rank 0 committed rounds past the coordinator's counter: the coordinator pulls
  that model, advances the round counter and rolls the survivors forward to it;
* two real client processes (gloo collective): a lease of 5 runs 5 rounds per StartTrain, per-round stats
  reach the coordinator's metrics, and every client ends on the persisted global model.
"""
import json
import time

import pytest
import torch

from fedmi import ckpt as ck
from fedmi.control.coordinator import Coordinator, CoordinatorConfig
from fedmi.utils.metrics import MetricsLog
from fedmi.wire import proto as P

import subprocess
import sys
from pathlib import Path

from fake_client import FakeClient, serve
from helpers import free_port, stop_proc


def _serve(n, **kw):
    """n in-process fake clients (tests/fake_client.py) on real gRPC servers."""
    fakes, servers, addrs = [], [], []
    for _ in range(n):
        f = FakeClient(**kw)
        srv, port = serve(f)
        fakes.append(f)
        servers.append(srv)
        addrs.append(f"127.0.0.1:{port}")
    return fakes, servers, addrs


def _spawn_fakes(tmp_path, n):
    """n fake client PROCESSES (their gRPC servers do not share the coordinator's interpreter)."""
    procs, addrs = [], []
    for i in range(n):
        pf = tmp_path / f"fake{i}.port"
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).with_name("fake_client.py")), str(pf)],
                                      stdout=subprocess.DEVNULL, stderr=subprocess.STDOUT, start_new_session=True))
    for i in range(n):
        pf = tmp_path / f"fake{i}.port"
        t0 = time.time()
        while not pf.exists():
            if time.time() - t0 > 120:
                raise TimeoutError("fake client did not start")
            time.sleep(0.05)
        addrs.append(f"127.0.0.1:{int(pf.read_text())}")
    return procs, addrs


def _overhead_per_round(addrs, root, lease: int, rounds: int = 64) -> float:
    if True:
        cfg = CoordinatorConfig(clients=addrs, rounds=rounds, agg="collective", root=str(root),
                                rpc_timeout_s=10, train_timeout_s=30, heartbeat_s=5.0, lease_rounds=lease, lease_s=0,
                                ckpt_fetch_interval_s=0)
        coord = Coordinator(cfg)
        coord.run_round()                        # warm the channels (first call carries the connection setup)
        t0 = time.perf_counter()
        while coord.round < rounds:
            assert coord.run_round()
        dt = (time.perf_counter() - t0) / (rounds - (lease if lease > 1 else 1))
        coord.close()
        return dt * 1e3


def test_lease_amortises_the_round_trip_flat_in_clients(tmp_path):
    """Coordinator-side cost per round (no training: everything measured is control plane).  With a
    16-round lease it is a fraction of the one-RPC-per-round cadence at every client count, and it does
    not grow with the number of clients beyond the per-lease fan-out."""
    rows = {}
    procs, addrs = _spawn_fakes(tmp_path, 8)
    try:
        for n in (1, 2, 4, 8):
            rows[n] = (_overhead_per_round(addrs[:n], tmp_path / f"s{n}_1", 1),
                       _overhead_per_round(addrs[:n], tmp_path / f"s{n}_16", 16))
    finally:
        for p in procs:
            stop_proc(p)
    print("per-round control-plane ms (lease 1, lease 16):", {n: tuple(round(v, 3) for v in r) for n, r in rows.items()})
    for n, (one, leased) in rows.items():
        assert leased < 0.35 * one, (n, one, leased)
    # what is left per round is the per-lease fan-out / 16: at 8 clients a small constant (this container's
    # bare gRPC round trip is ~3 ms; the per-round-RPC cadence pays it N times every round)
    assert rows[8][1] < 3.0 and rows[8][1] < 0.25 * rows[8][0], rows


def test_aborted_lease_advances_to_rank0_committed_round(tmp_path):
    """A lease that fails at round r after rank 0 committed rounds up to r-1 (> the coordinator's counter):
    the coordinator installs rank 0's committed model, advances its round counter to that epoch, rolls
    every surviving member forward to it, and numbers the next round epoch + 1."""
    fakes, servers, addrs = _serve(2)
    try:
        cfg = CoordinatorConfig(clients=addrs, rounds=40, agg="collective", root=str(tmp_path / "srv"),
                                rpc_timeout_s=10, train_timeout_s=30, heartbeat_s=5.0, lease_rounds=8, lease_s=0,
                                ckpt_fetch_interval_s=0)
        coord = Coordinator(cfg)
        assert coord.run_round() and coord.round == 8
        for f in fakes:                          # next lease (rounds 9-16) fails at round 12: 9-11 committed
            f.abort_at = (12, 11)
        assert not coord.run_round()
        assert coord.round == 11 and coord.installed_epoch == 11
        assert all(f.installed[-1:] == [11] for f in fakes), [f.installed for f in fakes]
        for f in fakes:
            f.abort_at = None
        seen = []
        orig = coord._meta

        def spy(rnd, live, lease=1):
            seen.append((rnd, lease))
            return orig(rnd, live, lease)

        coord._meta = spy
        assert coord.run_round()
        assert seen[0][0] == 12 and coord.round == 11 + seen[0][1]
        coord.close()
    finally:
        for s in servers:
            s.stop(grace=0)


def test_single_round_abort_with_rank0_ahead(tmp_path):
    """lease 1 (reference cadence): rank 0's ABORTED trailer and fetch report epoch round + 1 -- its all-reduce
    finished before another client died -- so that model is committed and the counter advances to it."""
    fakes, servers, addrs = _serve(2)
    try:
        cfg = CoordinatorConfig(clients=addrs, rounds=20, agg="collective", root=str(tmp_path / "srv"),
                                rpc_timeout_s=10, train_timeout_s=30, heartbeat_s=5.0, lease_rounds=1,
                                ckpt_fetch_interval_s=0)
        coord = Coordinator(cfg)
        for _ in range(3):
            assert coord.run_round()
        assert coord.round == 3
        for f in fakes:
            f.abort_at = (4, 4)                  # round 4 "aborted" but rank 0 committed it
        assert not coord.run_round()
        assert coord.round == 4 and coord.installed_epoch == 4
        assert all(f.installed[-1] == 4 for f in fakes)
        for f in fakes:
            f.abort_at = None
        assert coord.run_round() and coord.round == 5
        coord.close()
    finally:
        for s in servers:
            s.stop(grace=0)


def test_nonzero_rank_lost_after_final_round_keeps_rank0_lease(tmp_path):
    """rank 0 finished the whole lease and replied OK, a non-zero rank died after the last collective
    (UNAVAILABLE before its reply landed).  Every round of the lease completed its all-reduce, so the coordinator
    commits up to rank 0's round instead of rolling every survivor back a whole lease; the loss is propagated to
    the generation's store (abort key) at once."""
    fakes, servers, addrs = _serve(2)
    try:
        metrics = MetricsLog(tmp_path / "coord.jsonl")
        cfg = CoordinatorConfig(clients=addrs, rounds=40, agg="collective", root=str(tmp_path / "srv"),
                                rpc_timeout_s=10, train_timeout_s=30, heartbeat_s=5.0, lease_rounds=8, lease_s=0,
                                ckpt_fetch_interval_s=0)
        coord = Coordinator(cfg, metrics=metrics)
        assert coord.run_round() and coord.round == 8
        gen = coord.generation
        fakes[1].lost_after_lease = True         # rounds 9-16 all run on both, then rank 1 dies
        assert not coord.run_round()
        assert coord.round == 16 and coord.installed_epoch == 16, (coord.round, coord.installed_epoch)
        assert fakes[0].installed[-1:] == [16], fakes[0].installed          # rolled to rank 0's round, not to 8
        assert coord.client_status()[addrs[1]] is False
        assert coord.store.store.check([f"fedmi/gen{gen}/abort"])        # survivors' watchdogs see the loss
        metrics.flush()
        ev = [json.loads(x) for x in (tmp_path / "coord.jsonl").read_text().splitlines()]
        assert [r["client"] for r in ev if r.get("event") == "loss_propagated"] == [addrs[1]]
        seen = []
        orig = coord._meta
        coord._meta = lambda rnd, live, lease=1: (seen.append(rnd), orig(rnd, live, lease))[1]
        assert coord.run_round() and seen[0] == 17
        coord.close()
    finally:
        for s in servers:
            s.stop(grace=0)


def test_lease_deadline_follows_round_time(tmp_path):
    """a lease's StartTrain deadline is the per-round timeout plus the lease's expected run time, not
    lease x the per-round timeout (a stuck-but-alive client would otherwise hold a 64-round lease for hours)."""
    cfg = CoordinatorConfig(clients=[], rounds=10, agg="grpc", root=str(tmp_path / "srv"), train_timeout_s=600)
    coord = Coordinator(cfg)
    try:
        assert coord._train_deadline(1) == 600
        coord._round_s = 0.01
        assert coord._train_deadline(64) == pytest.approx(600 + 4 * 64 * 0.01)
        coord._round_s = None
        assert coord._train_deadline(4) == 2400          # no measured round yet: the old bound
    finally:
        coord.close()


def test_rollback_below_rank0_checkpoint_resets_upload_buffer(tmp_path):
    """rank 0 serialised rounds up to 5, then the coordinator rolls it back to round 3 (SendModel).  The
    fetch path must serve the installed round-3 model (nothing newer than have=3), and after the re-run round 4 the
    fetched model is the NEW round 4 -- never the abandoned branch's round 5 labelled with a higher epoch."""
    from fedmi.control.client_agent import META_FETCH, META_HAVE, META_LEASE, META_ROUND, ClientAgent, serve_client
    from helpers import small_trainer

    addr = f"127.0.0.1:{free_port()}"
    ag = ClientAgent(small_trainer("mlp", seed=0), addr, root=tmp_path / "c0", agg="collective", verbose=False)
    srv, _ = serve_client(ag, addr)
    stub = P.TrainerStub(P.make_channel(addr))

    def fetch(have):
        reply, call = stub.SendModel.with_call(P.SendModelRequest(model=""), timeout=30,
                                               metadata=[(META_FETCH, "1"), (META_HAVE, str(have))])
        return int(dict(call.trailing_metadata())["x-fedmi-ckpt-epoch"]), reply.reply

    try:
        stub.StartTrain(P.TrainRequest(rank=0, world=1), timeout=120, metadata=[(META_ROUND, "1"), (META_LEASE, "3")])
        committed3 = ck.to_bytes(ck.make_checkpoint(ag.trainer.state_dict(), acc=1, epoch=3))
        stub.StartTrain(P.TrainRequest(rank=0, world=1), timeout=120, metadata=[(META_ROUND, "4"), (META_LEASE, "2")])
        ag.writer.flush()
        assert fetch(-1)[0] == 5
        stub.SendModel(P.SendModelRequest(model=ck.to_b64(committed3)), timeout=60)        # rollback to round 3
        epoch, b64 = fetch(3)
        assert epoch == 3 and b64 == "", epoch                       # not the abandoned round 5
        stub.StartTrain(P.TrainRequest(rank=0, world=1), timeout=120, metadata=[(META_ROUND, "4")])
        ag.writer.flush()
        epoch, b64 = fetch(3)
        assert epoch == 4 and b64
        got = ck.from_bytes(ck.from_b64(b64))["net"]
        assert ck.state_digest(got) == ck.state_digest(ag.trainer.state_dict())
    finally:
        srv.stop(None)
        ag.close()


@pytest.mark.slow
def test_lease_with_real_clients(tmp_path):
    from helpers import spawn_client, wait_heartbeat

    addrs = [f"127.0.0.1:{free_port()}" for _ in range(2)]
    procs = [spawn_client(a, tmp_path, "--agg", "collective", "--model", "mlp", "--data", "synthetic-mnist",
                          "--n-train", "512", "--n-test", "256", "--backend", "gloo", "--lr", "0.05",
                          log_path=tmp_path / f"client{i}.log") for i, a in enumerate(addrs)]
    try:
        for a in addrs:
            wait_heartbeat(a, timeout=120)
        metrics = MetricsLog(tmp_path / "primary.jsonl")
        cfg = CoordinatorConfig(clients=addrs, rounds=12, agg="collective", root=str(tmp_path / "srv"),
                                train_timeout_s=120, rpc_timeout_s=10, heartbeat_s=0.2, lease_rounds=5, lease_s=0)
        coord = Coordinator(cfg, metrics=metrics)
        calls = []
        orig = coord._meta
        coord._meta = lambda rnd, live, lease=1: (calls.append((rnd, lease)), orig(rnd, live, lease))[1]
        coord.run()
        coord.close()
        metrics.close()
        assert calls == [(1, 5), (6, 5), (11, 2)]
        assert coord.round == 12
        rows = [json.loads(x) for x in (tmp_path / "primary.jsonl").read_text().splitlines()]
        rounds = [r for r in rows if r.get("event") == "round"]
        assert [r["round"] for r in rounds] == list(range(1, 13))
        assert all(r["ok"] and "train_loss" in r and r["test_acc"] > 0 for r in rounds)
        g = ck.load(tmp_path / "srv" / "Primary" / "optimizedModel.pth")
        assert g["epoch"] == 12
        for a in addrs:
            c = ck.load(tmp_path / "checkpoint" / f"{a}.pth")
            assert c["epoch"] == 12
            for k in g["net"]:
                assert torch.allclose(c["net"][k], g["net"][k], atol=1e-6), k
    finally:
        for p in procs:
            stop_proc(p)


def test_lease_length_follows_round_time(tmp_path):
    """cfg.lease_s: the first StartTrain covers one round (the round time is unknown), then the lease covers
    about lease_s of rounds -- ~10 ms rounds get long leases (capped at lease_rounds), rounds slower than lease_s
    keep one StartTrain per round (the coordinator reacts at that cadence)."""
    def leases(work_s, lease_s, cap, rounds):
        fakes, servers, addrs = _serve(1, work_s=work_s)
        try:
            cfg = CoordinatorConfig(clients=addrs, rounds=rounds, agg="collective", root=str(tmp_path / f"s{work_s}"),
                                    rpc_timeout_s=10, train_timeout_s=30, heartbeat_s=5.0, lease_rounds=cap,
                                    lease_s=lease_s, ckpt_fetch_interval_s=0)
            coord = Coordinator(cfg)
            seen = []
            orig = coord._meta
            coord._meta = lambda rnd, live, lease=1: (seen.append(lease), orig(rnd, live, lease))[1]
            while coord.round < rounds:
                assert coord.run_round()
            coord.close()
            return seen
        finally:
            for s in servers:
                s.stop(grace=0)

    fast = leases(0.005, 0.1, 64, 120)              # ~5-6 ms rounds: ~16-20 rounds per lease
    # (the first rounds run slower -- warm-up, a loaded CPU under xdist -- so the lease ramps up over a few
    # StartTrains; never past lease_s / work_s = 20 since no round beats work_s)
    mid = sorted(fast[1:-1])[len(fast[1:-1]) // 2]
    assert fast[0] == 1 and 8 <= mid <= 20 and max(fast) <= 20, fast
    capped = leases(0.002, 1.0, 12, 60)             # a long target is capped at lease_rounds
    assert capped[0] == 1 and max(capped) == 12, capped
    slow = leases(0.03, 0.02, 64, 6)                # rounds slower than the target: one round per StartTrain
    assert slow == [1] * 6, slow
