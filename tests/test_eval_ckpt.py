"""Data-parallel evaluation (test set split over clients, accumulators summed in
one collective) equals the reference's every-client-evaluates-everything
(src/client.py:30 -> src/main.py:167-191); coalesced checkpoint snapshots keep
the reference file format (one storage per tensor, src/main.py:160-165)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import free_port, small_trainer


def test_eval_shard_covers_test_set():
    from fedmi.engine.data import ImageSet
    from fedmi.parallel.fedavg import eval_shard

    n = 1003
    s = ImageSet(torch.zeros(n, 1, 2, 2, dtype=torch.uint8), torch.arange(n, dtype=torch.int32))
    for w in (1, 2, 3, 8):
        ys = torch.cat([eval_shard(s, r, w).y for r in range(w)])
        assert torch.equal(ys, s.y)


def test_eval_history_single_rank():
    from fedmi.parallel.fedavg import EvalHistory

    tr = small_trainer("mlp", n_train=256, n_test=200)
    h = EvalHistory(tr, 3)
    ref = []
    for _ in range(3):
        tr.evaluate()
        h.record()
        ref.append(tr.eval_stats())
        tr.set_schedule([0], [128])
        tr.train_epoch()
    got = h.reduce()
    assert [g.count for g in got] == [200] * 3
    for g, r in zip(got, ref):
        assert g.correct == r.correct and g.loss_sum == pytest.approx(r.loss_sum, rel=1e-12)
    with pytest.raises(IndexError):
        h.record()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fedmi.parallel.fedavg import EvalHistory, eval_shard

    tr = small_trainer("mlp", n_train=128, n_test=301, seed=5)     # same seed -> same model on both ranks
    full = small_trainer("mlp", n_train=128, n_test=301, seed=5)
    tr.set_test_data(eval_shard(tr.test_set, rank, world))
    h = EvalHistory(tr, 2)
    for _ in range(2):
        tr.evaluate()
        h.record()
    got = h.reduce()
    full.evaluate()
    q.put((rank, [(g.loss_sum, g.correct, g.count) for g in got], full.eval_stats()))
    dist.destroy_process_group()


@pytest.mark.slow
def test_sharded_eval_equals_full_eval_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, f)) for r, g, f in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        got, full = res[r]
        for loss_sum, correct, count in got:
            assert count == full.count == 301
            assert correct == full.correct
            assert loss_sum == pytest.approx(full.loss_sum, rel=1e-6)   # fp32 batch sums, other order


def test_async_writer_coalesced_views(tmp_path):
    from fedmi.ckpt import AsyncCheckpointWriter, load

    flat = torch.arange(30, dtype=torch.float32)
    sd = {"a.weight": flat[0:12].view(3, 4), "a.bias": flat[12:15], "b.weight": flat[15:30].view(5, 3),
          "bn.num_batches_tracked": torch.tensor(7, dtype=torch.int64)}
    w = AsyncCheckpointWriter()
    paths = [tmp_path / "Primary" / "optimizedModel.pth", tmp_path / "checkpoint" / "c0.pth"]
    w.submit(paths, sd, acc=1, epoch=4)
    w.close()
    for p in paths:
        ck = load(p)
        assert ck["epoch"] == 4 and ck["acc"] == 1
        assert list(ck["net"]) == list(sd)
        for k, v in sd.items():
            assert torch.equal(ck["net"][k], v)
        assert ck["net"]["a.bias"].untyped_storage().nbytes() == 12    # own storage, like module.state_dict()
