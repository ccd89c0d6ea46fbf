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


def test_async_writer_coalesces_superseded_rounds(tmp_path, monkeypatch):
    """A writer slower than the round cadence keeps only the newest queued checkpoint per file
    set: submit never blocks, flush leaves the LAST round on disk, and other files keep FIFO."""
    import threading

    import fedmi.ckpt as ck

    gate = threading.Event()
    real = ck.atomic_write
    order = []

    def slow_write(path, data):
        gate.wait(10)
        order.append(path.name)
        real(path, data)

    monkeypatch.setattr(ck, "atomic_write", slow_write)
    w = ck.AsyncCheckpointWriter(max_pending=2)
    a, b = tmp_path / "a.pth", tmp_path / "b.pth"
    t = torch.zeros(4)
    w.submit(a, {"w": t + 0}, epoch=0)            # picked up by the writer, blocked in the write
    import time
    deadline = time.monotonic() + 5
    while not w._busy and time.monotonic() < deadline:
        time.sleep(0.001)
    for r in range(1, 50):                        # 49 more rounds: would block on a 2-deep queue
        w.submit(a, {"w": t + r}, epoch=r)
    w.submit(b, {"w": t - 1}, epoch=7)
    assert w.coalesced == 48
    gate.set()
    w.flush()
    assert ck.load(a)["epoch"] == 49 and torch.equal(ck.load(a)["net"]["w"], t + 49)
    assert ck.load(b)["epoch"] == 7
    assert order == ["a.pth", "a.pth", "b.pth"]
    w.close()


def test_async_writer_no_coalesce_writes_every_submission(tmp_path, monkeypatch):
    import fedmi.ckpt as ck

    seen = []
    real = ck.atomic_write
    monkeypatch.setattr(ck, "atomic_write", lambda p, d: (seen.append(ck.from_bytes(d)["epoch"]), real(p, d)))
    w = ck.AsyncCheckpointWriter(max_pending=2, coalesce=False)
    for r in range(10):
        w.submit(tmp_path / "a.pth", {"w": torch.full((3,), float(r))}, epoch=r)
    w.close()
    assert seen == list(range(10))


def test_native_round_writer_matches_torch_save(tmp_path):
    """The C++ writer's archives (host mode on CPU) load with weights_only torch.load, pass the
    zip CRC check, hold the newest round after flush, and coalesce rounds it could not keep up with."""
    import zipfile
    from collections import OrderedDict

    from fedmi import native
    from fedmi.ckpt import RoundCheckpointWriter, load

    if not native.available():
        pytest.skip("native extension not built")
    flat = torch.randn(64)
    nbt = torch.tensor(5, dtype=torch.int64)
    sd = OrderedDict([("module.a.weight", flat[0:12].view(3, 4)), ("a.bias", flat[12:15]),
                      ("bn.num_batches_tracked", nbt), ("b.weight", flat[20:35].view(5, 3)),
                      ("empty", flat[40:40])])
    paths = [tmp_path / "Primary" / "optimizedModel.pth", tmp_path / "checkpoint" / "c0.pth"]
    w = RoundCheckpointWriter(coalesce=True, slots=2)
    for r in range(100):
        flat.add_(1.0)
        nbt.add_(1)
        w.submit(paths, sd, acc=1, epoch=r + 1 if r < 99 else 70000)   # last epoch needs all 4 bytes
    w.flush()
    assert w.backend == "native"
    assert w.written + 2 * w.coalesced == 200
    for p in paths:
        assert zipfile.ZipFile(p).testzip() is None
        ck = load(p)
        assert ck["epoch"] == 70000 and ck["acc"] == 1
        assert list(ck["net"]) == ["a.weight", "a.bias", "bn.num_batches_tracked", "b.weight", "empty"]
        for k, v in sd.items():
            assert torch.equal(ck["net"][k.replace("module.", "")], v)
        assert ck["net"]["bn.num_batches_tracked"].dtype == torch.int64
    # a different acc rebuilds the template; a new state-dict layout rebuilds the writer
    w.submit(paths, sd, acc=0.5, epoch=3)
    sd2 = OrderedDict([("x", torch.ones(2, 2))])
    w.submit(paths[:1], sd2, acc=1, epoch=4)
    w.close()
    assert load(paths[1])["acc"] == 0.5 and load(paths[1])["epoch"] == 3
    assert list(load(paths[0])["net"]) == ["x"] and load(paths[0])["epoch"] == 4


def test_native_round_writer_writes_every_round_in_order(tmp_path, monkeypatch):
    """Default (no coalescing): every submitted round reaches the disk, in order."""
    from fedmi import native
    from fedmi.ckpt import RoundCheckpointWriter, load

    if not native.available():
        pytest.skip("native extension not built")
    flat = torch.zeros(1000)
    sd = {"w": flat[:600].view(20, 30), "b": flat[600:]}
    w = RoundCheckpointWriter(slots=2)
    seen = []
    for r in range(60):
        flat.fill_(float(r))
        w.submit(tmp_path / "m.pth", sd, epoch=r)
        if r % 7 == 0:
            w.flush()
            seen.append(load(tmp_path / "m.pth")["epoch"])
    w.close()
    assert w.coalesced == 0 and w.written == 60
    assert seen == [r for r in range(60) if r % 7 == 0]
    ck = load(tmp_path / "m.pth")
    assert ck["epoch"] == 59 and torch.equal(ck["net"]["w"], torch.full((20, 30), 59.0))


def test_native_writer_targets_are_independent_files(tmp_path):
    """Default: Primary/optimizedModel.pth and checkpoint/<client>.pth are separate inodes, so a peer that
    rewrites one of them IN PLACE (the reference's torch.save: truncate + write, src/server.py:179) leaves
    the other intact.  ``link=True`` (opt-in) shares one inode."""
    import os

    from fedmi import native
    from fedmi.ckpt import RoundCheckpointWriter, load

    if not native.available():
        pytest.skip("native extension not built")
    sd = {"w": torch.arange(12.0).view(3, 4)}
    paths = [tmp_path / "Primary" / "optimizedModel.pth", tmp_path / "checkpoint" / "c0.pth"]
    w = RoundCheckpointWriter(slots=2)
    for r in range(3):
        w.submit(paths, sd, epoch=r + 1)
    w.close()
    assert w.backend == "native"
    assert os.stat(paths[0]).st_ino != os.stat(paths[1]).st_ino
    with open(paths[0], "r+b") as f:     # in-place rewrite of one target
        f.truncate(0)
        f.write(b"garbage")
    ck = load(paths[1])
    assert ck["epoch"] == 3 and torch.equal(ck["net"]["w"], sd["w"])
    lk = RoundCheckpointWriter(slots=2, link=True)
    lp = [tmp_path / "own" / "a.pth", tmp_path / "own" / "b.pth"]
    lk.submit(lp, sd, epoch=7)
    lk.close()
    assert os.stat(lp[0]).st_ino == os.stat(lp[1]).st_ino and load(lp[1])["epoch"] == 7


@pytest.mark.gpu
def test_device_round_writer_native_vs_python(tmp_path, monkeypatch):
    """Device tensors: the native writer (default) and the Python writer (FEDMI_NATIVE_CKPT=0) produce
    archives with the same contents, and each round's file holds the values as of ITS submit even though
    the stream overwrites the tensors right after (the snapshot copy is stream-ordered)."""
    from fedmi.ckpt import RoundCheckpointWriter, load

    dev = torch.device("cuda", 0)
    flat = torch.zeros(62006, device=dev)
    sd = {"w": flat[:50000].view(100, 500), "b": flat[50000:]}
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("FEDMI_NATIVE_CKPT", mode)
        w = RoundCheckpointWriter(slots=3)
        seen = []
        for r in range(12):
            flat.fill_(float(r))
            w.submit(tmp_path / f"m{mode}.pth", sd, epoch=r)
            flat.add_(1000.0)           # enqueued after the snapshot: must not leak into round r's file
            if r % 4 == 3:
                w.flush()
                ck = load(tmp_path / f"m{mode}.pth")
                seen.append((ck["epoch"], float(ck["net"]["w"][0, 0]), float(ck["net"]["b"][-1])))
        w.close()
        assert w.backend == ("native" if mode == "1" else "python")
        out[mode] = seen
    assert out["1"] == out["0"] == [(r, float(r), float(r)) for r in (3, 7, 11)]
