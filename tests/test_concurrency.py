"""Race detection on the control plane: a client agent under concurrent RPC load.

While a coordinator thread drives StartTrain rounds, other threads hammer the same agent with
checkpoint fetches (SendModel + x-fedmi-fetch), heartbeats and StartTrain calls from a STALE term,
and a fourth thread keeps re-reading the persisted checkpoint.  Every call runs under a deadline
(a deadlock fails the test instead of hanging it).  Checked: no unexpected RPC error, stale terms
are fenced, fetched and persisted epochs never go backwards, and the final state is consistent.
"""
import threading
import time

import grpc
import pytest

from fedmi import ckpt as ck
from fedmi.control.client_agent import META_FETCH, META_GEN, META_ROUND, META_TERM, ClientAgent, serve_client
from fedmi.wire import proto as P

from helpers import free_port, small_trainer

pytestmark = pytest.mark.timeout(180)


def test_client_agent_under_concurrent_rpcs(tmp_path):
    addr = f"127.0.0.1:{free_port()}"
    agent = ClientAgent(small_trainer(), addr, root=tmp_path, agg="collective", verbose=False)   # world 1, no group
    server = serve_client(agent, addr)[0]
    stub = P.TrainerStub(P.make_channel(addr))
    term = 10_000
    stop = threading.Event()
    errors, fetched, persisted, fenced = [], [], [], []
    rounds = 12

    def coordinator():
        try:
            for r in range(1, rounds + 1):
                md = [(META_TERM, str(term)), (META_ROUND, str(r)), (META_GEN, "1")]
                stub.StartTrain(P.TrainRequest(rank=0, world=1), timeout=60, metadata=md)
        except Exception as e:              # noqa: BLE001 -- reported below
            errors.append(("coordinator", repr(e)))
        finally:
            stop.set()

    def fetcher():
        while not stop.is_set():
            try:
                reply, call = stub.SendModel.with_call(P.SendModelRequest(model=""), timeout=10,
                                                       metadata=[(META_TERM, str(term)), (META_FETCH, "1")])
                ep = int(dict(call.trailing_metadata()).get("x-fedmi-ckpt-epoch", "-1"))
                fetched.append(ep)
            except grpc.RpcError as e:
                errors.append(("fetch", e.code().name))

    def heartbeats():
        while not stop.is_set():
            try:
                assert stub.HeartBeat(P.Request(), timeout=5).status == 1
            except Exception as e:          # noqa: BLE001
                errors.append(("heartbeat", repr(e)))

    def stale_coordinator():
        while agent.max_term < term and not stop.is_set():     # once the new term is known,
            time.sleep(0.001)                                   # EVERY older-term call must be fenced
        while not stop.is_set():
            try:
                stub.StartTrain(P.TrainRequest(rank=0, world=1), timeout=60,
                                metadata=[(META_TERM, str(term - 1)), (META_ROUND, "1"), (META_GEN, "1")])
                errors.append(("stale", "a stale-term StartTrain was accepted after the new term"))
            except grpc.RpcError as e:
                if e.code() == grpc.StatusCode.FAILED_PRECONDITION:
                    fenced.append(1)
                else:
                    errors.append(("stale", e.code().name))
            time.sleep(0.01)

    def reader():
        path = agent.ckpt_path
        while not stop.is_set():
            if path.exists():
                try:
                    persisted.append(int(ck.load(path)["epoch"]))
                except Exception as e:      # noqa: BLE001 -- a torn file would land here
                    errors.append(("reader", repr(e)))
            time.sleep(0.005)

    threads = [threading.Thread(target=f, daemon=True) for f in (fetcher, heartbeats, stale_coordinator, reader)]
    main = threading.Thread(target=coordinator, daemon=True)
    for t in threads:
        t.start()
    time.sleep(0.05)
    main.start()
    main.join(timeout=150)
    stop.set()
    for t in threads:
        t.join(timeout=20)
    try:
        assert not main.is_alive() and not any(t.is_alive() for t in threads), "deadlock: a thread never returned"
        assert not errors, errors[:5]
        assert agent.round == rounds
        assert fenced, "the stale coordinator was never fenced"
        assert fetched and max(fetched) > 0, "no checkpoint was ever fetched"
        assert all(b >= a for a, b in zip(fetched, fetched[1:])), "fetched epochs went backwards"
        assert all(b >= a for a, b in zip(persisted, persisted[1:])), "persisted epochs went backwards"
        agent.writer.flush()
        assert ck.load(agent.ckpt_path)["epoch"] == rounds
    finally:
        server.stop(grace=None)
        agent.close()
