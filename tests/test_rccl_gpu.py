"""The RCCL (``nccl`` backend) data-plane lifecycle on this ROCm build, at world 1.

RCCL refuses two ranks on one GPU, so a one-GPU box can only run a 1-rank
communicator -- but that already executes every call the multi-GPU path makes:
``GroupManager("nccl", transport="dist").ensure`` -> ``init_process_group``
(ncclCommInitRank over a generation-prefixed TCPStore) -> ``all_reduce(AVG)`` /
``broadcast`` / ``all_gather`` -> ``interrupt()`` (``_abort_process_group`` =
ncclCommAbort, the path a client takes when a newer membership generation
arrives mid-collective) -> ``ensure`` of the next generation (a fresh
communicator in the same process) -> collectives again.  The error-handling
environment of ``fedmi/cli/client.py`` (async error handling 3, blocking wait)
is set as in production.  Each case runs in its own spawned process so the
default process group never leaks into the test runner.
"""
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(180)]


def _lifecycle(q):
    import os

    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "3")
    os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
    import torch.distributed as dist

    from fedmi.parallel.fedavg import allreduce_int_mean_, allreduce_mean_
    from fedmi.parallel.group import GroupManager, Membership, StoreHost

    res = {"ok": True, "msgs": [], "backend": None}
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        host = StoreHost("127.0.0.1", 0)
        gm = GroupManager("nccl", dev, timeout_s=30.0, transport="dist", init_world1=True)
        for gen in (1, 2, 3):
            changed = gm.ensure(Membership(gen, 0, 1, "127.0.0.1", host.port))
            if not changed or not dist.is_initialized():
                res["ok"] = False
                res["msgs"].append(f"gen {gen}: ensure did not form a group")
                break
            res["backend"] = dist.get_backend()
            x = torch.arange(1 << 16, dtype=torch.float32, device=dev) * gen
            y = x.clone()
            dist.all_reduce(y, op=dist.ReduceOp.AVG)
            allreduce_mean_(y)                                     # world 1 -> identity
            b = torch.full((7,), float(gen), device=dev)
            dist.broadcast(b, src=0)
            outs = [torch.empty(5, device=dev)]
            dist.all_gather(outs, torch.full((5,), 3.0 * gen, device=dev))
            iv = torch.tensor([gen, -gen], dtype=torch.int64, device=dev)
            dist.all_reduce(iv, op=dist.ReduceOp.SUM)
            allreduce_int_mean_(iv)
            torch.cuda.synchronize()
            if not (torch.equal(x, y) and torch.equal(b, torch.full((7,), float(gen), device=dev))
                    and torch.equal(outs[0], torch.full((5,), 3.0 * gen, device=dev))
                    and iv.tolist() == [gen, -gen]):
                res["ok"] = False
                res["msgs"].append(f"gen {gen}: collective result mismatch")
            # same membership again: no regroup
            if gm.ensure(Membership(gen, 0, 1, "127.0.0.1", host.port)):
                res["ok"] = False
                res["msgs"].append(f"gen {gen}: unchanged membership regrouped")
            gm.interrupt()                                         # ncclCommAbort of the default group
            if dist.is_initialized():
                res["ok"] = False
                res["msgs"].append(f"gen {gen}: group still initialised after abort")
        gm.shutdown()
        res["generations"] = gm.generations_joined
    except Exception as e:  # pragma: no cover - reported to the parent
        res["ok"] = False
        res["msgs"].append(repr(e))
    q.put(res)


def test_rccl_init_allreduce_abort_regroup_world1():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_lifecycle, args=(q,))
    p.start()
    res = q.get(timeout=150)
    p.join(timeout=30)
    assert res["ok"], res["msgs"]
    assert res["backend"] == "nccl"
    assert res["generations"] == 3
    assert p.exitcode == 0
