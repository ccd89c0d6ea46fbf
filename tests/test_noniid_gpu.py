"""BASELINE config 3 parity: FedAvg of ResNet-18 over 2 non-IID clients (2 label shards each), the
native HIP engine vs plain PyTorch fp32, same split / init / recipe (lr 0.02, where the recipe is
stable; profiles/r3_noniid/README.md has the lr 0.1 sweep).  Both clients run in this process
(tools/fedavg_sim.py semantics: one local epoch each, uniform mean of the float state, floor mean of
num_batches_tracked, global model evaluated on the full test set)."""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.slow, pytest.mark.timeout(420)]


@pytest.fixture(autouse=True)
def _deterministic(deterministic_reference):
    """Every test here compares against the deterministic fp32 reference (conftest.deterministic_reference)."""
    yield


def _run(engine: str, rounds: int, monkeypatch, lr: float = 0.02, augment: bool = True, seed: int = 17,
         clients: int = 2, data_spec: str = "synthetic-cifar10", n_train: int = 50000, n_test: int = 10000):
    if engine == "fp32":
        monkeypatch.setenv("FEDMI_TORCH_PATH", "1")
    else:
        monkeypatch.delenv("FEDMI_TORCH_PATH", raising=False)
    from fedmi.engine import build_trainer
    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.data import contiguous_schedule, label_shard_indices, make_dataset

    dev = torch.device("cuda", 0)
    data = make_dataset(data_spec, device=dev, n_train=n_train, n_test=n_test, seed=0)
    cfg = TrainerConfig(seed=seed, lr=lr, augment=augment)
    W = clients
    shards = label_shard_indices(data.train.y.cpu().numpy(), W, 2, seed=0)
    clients, init = [], None
    for r in range(W):
        tr = build_trainer("resnet18", data, dev, cfg, init_state=init)
        if init is None:
            init = {k: v.detach().cpu().clone() for k, v in tr.state_dict().items()}
        tr.set_train_data(data.train.subset(shards[r]))
        tr.set_schedule(*contiguous_schedule(len(shards[r]), 128))
        clients.append(tr)
    accs, train_accs = [], []
    for _ in range(rounds):
        for tr in clients:
            tr.train_epoch()
        train_accs.append([tr.train_stats().acc for tr in clients])
        with torch.no_grad():
            mean = torch.stack([tr.float_state() for tr in clients]).mean(0)
            ints = [torch.div(sum(bs), W, rounding_mode="floor")
                    for bs in zip(*[[b.clone() for b in tr.int_state()] for tr in clients])]
            for tr in clients:
                tr.float_state().copy_(mean)
                for b, v in zip(tr.int_state(), ints):
                    b.copy_(v)
                tr.after_aggregate()
        clients[0].evaluate()
        accs.append(clients[0].eval_stats().acc)
    return accs, train_accs


def test_native_tracks_fp32_on_noniid_label_shards(monkeypatch):
    rounds = 5
    nat, nat_tr = _run("native", rounds, monkeypatch)
    ref, ref_tr = _run("fp32", rounds, monkeypatch)
    # both learn on the skewed split (chance is 10 %), and the native engine stays close to fp32
    assert ref[-1] > 30.0 and nat[-1] > 30.0, (nat, ref)
    assert abs(nat[-1] - ref[-1]) < 10.0, (nat, ref)
    for a, b in zip(nat_tr[-1], ref_tr[-1]):
        assert abs(a - b) < 5.0, (nat_tr, ref_tr)


def test_native_tracks_fp32_at_reference_lr_without_augmentation(monkeypatch):
    """The reference lr 0.1 on the same split.  With the reference's crop/flip augmentation this recipe kills
    local training in round 1 for most seeds in EVERY engine -- fp32 PyTorch, PyTorch autocast-bf16 and the
    native engine alike (profiles/r4_noniid/README.md: death rates over 10 seeds); without augmentation it is
    stable, and there the native engine must learn like fp32 (both clients well above their 5-class chance
    of ~20 % after two local epochs, and within 10 points of fp32 either way).  Two-sided again (round 4 made
    it one-sided after a run where the then non-deterministic fp32 reference landed 12 points low): the
    reference now runs PyTorch's deterministic algorithms (fixture above)."""
    rounds = 2
    nat, nat_tr = _run("native", rounds, monkeypatch, lr=0.1, augment=False)
    ref, ref_tr = _run("fp32", rounds, monkeypatch, lr=0.1, augment=False)
    ref2, ref2_tr = _run("fp32", rounds, monkeypatch, lr=0.1, augment=False)
    assert ref2_tr == ref_tr and ref2 == ref, (ref_tr, ref2_tr)       # the reference is run-to-run stable
    for a, b in zip(nat_tr[-1], ref_tr[-1]):
        assert a > 50.0 and b > 50.0, (nat_tr, ref_tr)
        assert abs(a - b) < 10.0, (nat_tr, ref_tr)


def test_config3_scale_global_model_learns(monkeypatch):
    """Config 3 at its client count: 8 clients x 2 label shards (each client sees ~2 classes), reduced size
    (16k training images, 2k test, 12 rounds, lr 0.02), on the high-contrast synthetic set.  On the default
    low-contrast set every engine's averaged model -- deterministic fp32 PyTorch included -- stays at chance for
    20 rounds at every lr from 0.002 to 0.1 (profiles/r5_noniid/README.md); here FedAvg's global model rises
    clearly above chance in both engines, and the native engine's late-round accuracy stays within 10 points of
    the deterministic fp32 reference (both engines are run-to-run deterministic, so this pins one outcome)."""
    kw = dict(clients=8, data_spec="synthetic-cifar10-easy", n_train=16000, n_test=2000, lr=0.02)
    rounds = 12
    nat, _ = _run("native", rounds, monkeypatch, **kw)
    ref, _ = _run("fp32", rounds, monkeypatch, **kw)
    print("native", nat, "fp32", ref)
    assert max(nat) > 20.0 and max(ref) > 20.0, (nat, ref)            # chance is 10 %
    late = rounds // 2
    mn, mr = sum(nat[late:]) / (rounds - late), sum(ref[late:]) / (rounds - late)
    assert abs(mn - mr) < 10.0, (mn, mr, nat, ref)
