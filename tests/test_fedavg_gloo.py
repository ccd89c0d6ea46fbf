"""Data-plane FedAvg semantics on CPU (gloo, 2 processes): dense mean of the flat
float state, floor-mean of integer buffers (reference float-mean + int64
truncation, src/server.py:163-171), broadcast init, and the -c Y compressors
(top-k with error feedback == dense when k = n; int8 within quantisation error)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import free_port

pytestmark = pytest.mark.slow


class _Stub:
    """Minimal LocalTrainer surface used by FedAvg / compressors."""

    def __init__(self, rank: int, n: int = 1000):
        g = torch.Generator().manual_seed(100 + rank)
        self.flat = torch.randn(n, generator=g)
        self.ints = [torch.tensor([10 + 3 * rank], dtype=torch.int64)]
        self.packs = 0

    def float_state(self):
        return self.flat

    def int_state(self):
        return self.ints

    def after_aggregate(self):
        self.packs += 1


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fedmi.parallel.compress import Int8Compressor, TopKCompressor
    from fedmi.parallel.fedavg import FedAvg, broadcast_state_

    out = {}
    # dense
    t = _Stub(rank)
    FedAvg().average(t)
    out["dense"] = t.flat.clone()
    out["int"] = int(t.ints[0])
    out["packs"] = t.packs
    # broadcast init
    b = _Stub(rank)
    broadcast_state_(b, 0)
    out["bcast"] = b.flat.clone()
    # top-k with k = n equals dense FedAvg of the deltas from a common anchor
    anchor = _Stub(0).flat.clone()
    tk = _Stub(rank)
    tk.flat.copy_(anchor)
    comp = TopKCompressor(tk, ratio=1.0)
    tk.flat.add_(torch.full_like(tk.flat, float(rank + 1)))   # local update
    FedAvg(compressor=comp).average(tk)
    out["topk_full"] = tk.flat.clone()
    # top-k 10%: untransmitted mass stays in the residual
    tk2 = _Stub(rank)
    tk2.flat.copy_(anchor)
    c2 = TopKCompressor(tk2, ratio=0.1)
    delta = torch.linspace(-1, 1, tk2.flat.numel()) * (rank + 1)
    tk2.flat.add_(delta)
    FedAvg(compressor=c2).average(tk2)
    out["topk_resid"] = float(c2.residual.abs().sum())
    out["topk_sent_nonzero"] = int((tk2.flat != anchor).sum())
    # int8
    i8 = _Stub(rank)
    i8.flat.copy_(anchor)
    c3 = Int8Compressor(i8)
    i8.flat.add_(delta)
    FedAvg(compressor=c3).average(i8)
    out["int8"] = i8.flat.clone()
    # warm-up: the first aggregation is dense FedAvg (full delta, residual empty), the second is top-k
    wu = _Stub(rank)
    wu.flat.copy_(anchor)
    c4 = TopKCompressor(wu, ratio=0.1, warmup=1)
    wu.flat.add_(delta)
    FedAvg(compressor=c4).average(wu)
    out["warm_dense"] = wu.flat.clone()
    out["warm_resid0"] = float(c4.residual.abs().sum())
    wu.flat.add_(delta)
    FedAvg(compressor=c4).average(wu)
    out["warm_resid1"] = float(c4.residual.abs().sum())
    out["warm_rounds"] = (c4.dense_rounds, c4.rounds)
    # tensors travel by value (numpy pickles): torch's fd-sharing reducer races the worker's exit
    q.put((rank, {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in out.items()}))
    dist.destroy_process_group()


def test_fedavg_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    res = {r: {k: (torch.from_numpy(v) if hasattr(v, "dtype") and not torch.is_tensor(v) and not isinstance(v, (int, float)) else v)
               for k, v in d.items()} for r, d in res.items()}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, b = _Stub(0).flat, _Stub(1).flat
    mean = (a + b) / 2
    for r in (0, 1):
        assert torch.allclose(res[r]["dense"], mean, atol=1e-6)
        assert res[r]["int"] == (10 + 13) // 2          # float mean 11.5 -> int64 truncation 11
        assert res[r]["packs"] == 1
        assert torch.equal(res[r]["bcast"], a)
        assert torch.allclose(res[r]["topk_full"], a + 1.5, atol=1e-5)   # mean of +1 and +2
        assert res[r]["topk_resid"] > 0
        n = a.numel()
        delta_mean = torch.linspace(-1, 1, n) * 1.5
        assert (res[r]["int8"] - (a + delta_mean)).abs().max() < 2.0 / 127 + 1e-6
    assert torch.equal(res[0]["int8"], res[1]["int8"])
    for r in (0, 1):
        assert torch.allclose(res[r]["warm_dense"], a + torch.linspace(-1, 1, a.numel()) * 1.5, atol=1e-5)
        assert res[r]["warm_resid0"] == 0 and res[r]["warm_resid1"] > 0
        assert tuple(res[r]["warm_rounds"]) == (1, 2)
