"""Client data sharding: the reference's strided batch assignment (src/main.py:141-145)
and the non-IID label-shard mode (BASELINE config 3; McMahan et al. shards)."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from fedmi.engine.data import contiguous_schedule, label_shard_indices, strided_schedule


@given(n=st.integers(1, 5000), batch=st.sampled_from([1, 7, 100, 128]), world=st.integers(1, 8))
@settings(max_examples=60, deadline=None)
def test_strided_schedule_partitions_batches_like_the_reference(n, batch, world):
    nb = -(-n // batch)
    owned = {}
    for rank in range(world):
        starts, sizes = strided_schedule(n, batch, rank, world)
        for s, z in zip(starts, sizes):
            i = s // batch
            assert (i + 1) % world == rank                  # src/main.py:142-145
            assert z == min(batch, n - s)
            assert i not in owned
            owned[i] = rank
    assert sorted(owned) == list(range(nb))                 # every batch trained exactly once per round


def test_strided_schedule_world1_rank0_owns_everything():
    starts, sizes = strided_schedule(50000, 128, 0, 1)
    assert len(starts) == 391 and sum(sizes) == 50000


def test_contiguous_schedule_covers_all():
    starts, sizes = contiguous_schedule(1000, 128)
    assert starts[0] == 0 and sum(sizes) == 1000 and sizes[-1] == 1000 - 7 * 128


@pytest.mark.parametrize("world,spc", [(2, 2), (4, 2), (8, 2), (8, 3), (5, 1)])
def test_label_shards_are_disjoint_cover_and_non_iid(world, spc):
    rng = np.random.default_rng(0)
    labels = rng.integers(0, 10, size=50000)
    shards = label_shard_indices(labels, world, spc, seed=3)
    assert len(shards) == world
    allidx = np.concatenate(shards)
    assert len(allidx) == len(labels) and len(np.unique(allidx)) == len(labels)   # disjoint + complete
    for ids in shards:
        assert np.all(np.diff(ids) > 0)                     # ascending, no duplicates
        counts = np.bincount(labels[ids], minlength=10)
        present = int((counts > 0).sum())
        # a label-sorted shard covers ~10/(world*spc) classes, plus partial classes at both ends
        assert present <= spc * (2 + -(-10 // (world * spc))), (present, counts)
        if world * spc >= 10:
            # dominated by few labels: the top-spc labels hold most of the client's data
            top = np.sort(counts)[::-1][:spc].sum()
            assert top >= 0.5 * len(ids)
    # sizes balanced to within one shard boundary
    sizes = [len(s) for s in shards]
    assert max(sizes) - min(sizes) <= spc


def test_label_shards_deterministic_per_seed():
    labels = np.repeat(np.arange(10), 100)
    a = label_shard_indices(labels, 4, 2, seed=1)
    b = label_shard_indices(labels, 4, 2, seed=1)
    c = label_shard_indices(labels, 4, 2, seed=2)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert not all(np.array_equal(x, y) for x, y in zip(a, c))


def test_label_shards_2_per_client_gives_2_labels_when_shards_align():
    # 10 classes x 100 samples, 5 clients x 2 shards = 10 shards of exactly one class each
    labels = np.repeat(np.arange(10), 100)
    shards = label_shard_indices(labels, 5, 2, seed=0)
    for ids in shards:
        assert len(np.unique(labels[ids])) == 2 and len(ids) == 200
