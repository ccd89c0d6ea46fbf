"""End-of-run FedAvg guard (fedmi/parallel/consistency.py) and the peer transport's
colocation agreement (fedmi/parallel/peer.py ``agree_any``), on CPU with gloo.

The guard is what makes bench.py's N>1 line trustworthy: every rank all-gathers
(transport error flag, blake2b digest of its flat model); one diverged client
or one timed-out peer barrier fails the run on EVERY rank.  Reference
semantics being guarded: one global model per round on every client
(src/server.py:144-179)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import free_port

pytestmark = pytest.mark.slow


class _Stub:
    def __init__(self, n: int = 257, seed: int = 7):
        g = torch.Generator().manual_seed(seed)
        self.flat = torch.randn(n, generator=g)
        self.ints = [torch.tensor(5, dtype=torch.int64), torch.tensor([3], dtype=torch.int64)]   # BN counters: 0-dim

    def float_state(self):
        return self.flat

    def int_state(self):
        return self.ints


class _Transport:
    def __init__(self, err: int):
        self.err = err

    def error(self):
        return self.err


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fedmi.parallel.consistency import check_consistency
    from fedmi.parallel.peer import agree_any

    out = {}
    # identical models, no transport error -> ok
    t = _Stub()
    out["same"] = check_consistency(t)
    # a client that skipped one round (last rank perturbed by one ulp) -> every rank sees the failure
    p = _Stub()
    if rank == world - 1:
        p.flat[3] = torch.nextafter(p.flat[3], torch.tensor(float("inf")))
    out["diverged"] = check_consistency(p)
    # integer buffer differs -> failure
    i = _Stub()
    if rank == 0:
        i.ints[0] += 1
    out["int_diverged"] = check_consistency(i)
    # a peer barrier timed out on one rank (its model may even match) -> failure everywhere
    out["transport_err"] = check_consistency(_Stub(), transport=_Transport(1 if rank == 1 else 0))
    # colocation agreement: only rank 0 and 1 share a GPU (3 ranks on 2 GPUs) -> all three gate
    store = dist.distributed_c10d._get_default_store()
    out["coloc_mixed"] = agree_any(store, "t/mixed", rank, world, rank < 2)
    out["coloc_none"] = agree_any(store, "t/none", rank, world, False)
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def results():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_identical_models_pass(results):
    for r, out in results.items():
        c = out["same"]
        assert c["ok"] and c["ranks"] == 3 and c["distinct_digests"] == 1 and c["transport_errors"] == [0, 0, 0]
    assert len({out["same"]["digest"] for out in results.values()}) == 1


def test_one_ulp_divergence_fails_on_every_rank(results):
    for out in results.values():
        assert not out["diverged"]["ok"] and out["diverged"]["distinct_digests"] == 2


def test_int_buffer_divergence_fails(results):
    for out in results.values():
        assert not out["int_diverged"]["ok"]


def test_transport_error_fails_on_every_rank(results):
    for out in results.values():
        c = out["transport_err"]
        assert not c["ok"] and c["transport_errors"] == [0, 1, 0] and c["distinct_digests"] == 1


def test_colocation_decision_is_uniform(results):
    # a per-rank decision let the co-located ranks wait in the host gate for a rank that never gates
    assert [results[r]["coloc_mixed"] for r in range(3)] == [True, True, True]
    assert [results[r]["coloc_none"] for r in range(3)] == [False, False, False]


def test_single_process_is_trivially_consistent():
    from fedmi.parallel.consistency import check_consistency, model_digest

    c = check_consistency(_Stub())
    assert c["ok"] and c["ranks"] == 1
    assert model_digest(_Stub()) == model_digest(_Stub()) != model_digest(_Stub(seed=8))
