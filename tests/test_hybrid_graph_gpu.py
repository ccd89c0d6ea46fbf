"""Hybrid engine: a captured-graph SGD step reproduces the eager step (fedmi/engine/torch_engine.py)."""
import pytest
import torch

from fedmi.engine.base import TrainerConfig
from fedmi.engine.data import contiguous_schedule, make_dataset
from fedmi.models import build_model

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["SimpleDLA", "EfficientNetB0"])
def test_hybrid_graph_matches_eager(gpu_device, name, monkeypatch):
    from fedmi.engine.torch_engine import TorchTrainer

    monkeypatch.setenv("FEDMI_HYBRID_GRAPH", "1")
    data = make_dataset("synthetic-cifar10-easy", device=gpu_device, n_train=512, n_test=200, seed=0)
    init = build_model(name).state_dict()
    runs = {}
    for graph in (False, True):
        tr = TorchTrainer(name, data, gpu_device, TrainerConfig(batch_size=128, lr=0.05, seed=3, use_graph=graph),
                          init_state=init, hybrid=True)
        assert tr.use_graph == graph
        tr.set_schedule(*contiguous_schedule(len(data.train), 128))
        tr.train_epoch()
        torch.cuda.synchronize()
        if graph:
            assert tr._graph is not None
        runs[graph] = (tr.float_state().clone(), tr.train_stats())
    (fe, se), (fg, sg) = runs[False], runs[True]
    assert se.count == sg.count == 512
    init_flat = TorchTrainer(name, data, gpu_device, TrainerConfig(seed=3), init_state=init).float_state()
    de, dg = fe - init_flat, fg - init_flat
    cos = float(torch.nn.functional.cosine_similarity(de, dg, dim=0))
    # EfficientNet's drop-connect draws different masks eager vs replayed: only the direction is compared
    assert cos > (0.9 if name == "SimpleDLA" else 0.5), cos
    assert abs(se.loss - sg.loss) < 0.05 * se.loss, (se.loss, sg.loss)


@pytest.mark.parametrize("name", ["SENet18", "EfficientNetB0", "RegNetY_400MF"])
def test_hybrid_default_graph_is_stable_at_reference_lr(gpu_device, name, monkeypatch):
    """The default hybrid engine replays a captured graph of the native step; the three models whose
    round-1 replay went NaN (autocast / ATen backend, profiles/hybrid_graph_nan_diag_r1.txt) train
    160 SGD steps at lr 0.1 with finite state."""
    from fedmi.engine import build_trainer

    monkeypatch.delenv("FEDMI_HYBRID_GRAPH", raising=False)
    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=128 * 40, n_test=200, seed=0)
    tr = build_trainer(name, data, gpu_device, TrainerConfig(lr=0.1, seed=1))
    assert tr.hybrid and tr.use_graph
    tr.set_schedule(*contiguous_schedule(len(data.train), 128))
    losses = []
    for _ in range(4):                      # 160 SGD steps
        tr.train_epoch()
        losses.append(tr.train_stats().loss)
    torch.cuda.synchronize()
    assert tr._graph is not None and not tr.mode.fallbacks
    assert all(v == v for v in losses) and torch.isfinite(tr.float_state()).all(), losses
    assert losses[-1] < losses[0], losses
