"""Native CNN engine (implicit-GEMM conv, depthwise, fused BN kernels) on the GPU.

Gradient-level parity of a deep bf16 network against fp32 is ill-conditioned at
random init (torch's OWN bf16 model reaches only cos 0.92 / 0.38 on the first
layer of ResNet-18 / MobileNet against fp32), so the kernels are checked one by
one in test_cnn_kernels_gpu.py, the schedule exactly (fp32 emulation) in
test_cnn_engine_wiring.py, and here the end-to-end behaviour:
  * loss and the last layers' gradients match fp32 torch;
  * the native engine trains like PyTorch's own engine (same data / init / lr);
  * a HIP-graph replay of the step equals the eager launch sequence.
"""
import pytest
import torch
import torch.nn.functional as F

from fedmi.engine.base import TrainerConfig
from fedmi.engine.data import augment_normalize, contiguous_schedule, make_dataset
from fedmi.models import build_model

pytestmark = pytest.mark.gpu


def _cos(a, b):
    return float(F.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0))


@pytest.mark.parametrize("name,tail", [("ResNet18", ["linear.weight", "layer4.1.bn2.weight", "layer4.1.conv2.weight"]),
                                       ("ResNet50", ["linear.weight", "layer4.2.bn3.weight"]),
                                       ("MobileNet", ["linear.weight", "layers.12.bn2.weight"]),
                                       ("MobileNetV2", ["linear.weight", "bn2.weight"]),
                                       ("VGG11", ["classifier.weight", "features.26.weight", "features.25.weight"]),
                                       ("PreActResNet18", ["linear.weight", "layer4.1.conv2.weight",
                                                           "layer4.1.bn2.weight"]),
                                       ("GoogLeNet", ["linear.weight", "b5.b1.1.weight", "b5.b4.2.weight"])])
def test_loss_and_tail_grads_match_torch(gpu_device, name, tail):
    from fedmi.engine.cnn_native import CNNNativeTrainer

    nb = 64
    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=128, n_test=64, seed=0)
    tr = CNNNativeTrainer(name, data, gpu_device, TrainerConfig(batch_size=nb, augment=False, use_graph=False))
    init = {k: v.detach().clone() for k, v in tr.state_dict().items()}
    tr.grads_for_batch(0, nb)
    tr.stats.zero_()
    tr.grads_for_batch(0, nb)      # second pass: BN statistics shifted by the first pass's batch mean
    torch.cuda.synchronize()
    ref = build_model(name).to(gpu_device)
    ref.load_state_dict(init)
    ref.train()
    x = augment_normalize(data.train.x[:nb], None, 0, 0)
    with torch.no_grad():
        ref(x)
    loss = F.cross_entropy(ref(x), data.train.y[:nb].long())
    loss.backward()
    st = tr.train_stats()
    assert st.count == nb
    assert abs(st.loss - float(loss.detach())) < 0.02 * float(loss.detach())
    ours = dict(tr.model.named_parameters())
    refp = dict(ref.named_parameters())
    for k in tail:
        assert _cos(ours[k].grad, refp[k].grad) > 0.95, k
    # every gradient is finite and of the right scale
    for k, p in refp.items():
        g = ours[k].grad
        assert torch.isfinite(g).all(), k
    rs = dict(tr.model.named_buffers())
    for k, b in ref.named_buffers():
        if b.is_floating_point():
            assert torch.allclose(rs[k], b, rtol=5e-2, atol=5e-3), k
        else:
            assert int(rs[k]) == int(b), k


@pytest.mark.parametrize("name", ["ResNet18", "MobileNet", "MobileNetV2", "VGG11", "PreActResNet18", "GoogLeNet"])
def test_engine_is_deterministic(gpu_device, name):
    """Two engines from the same init on the same batch produce bit-identical gradients, batch statistics and
    running stats.  Every split-K / weight-gradient / head reduction is fixed-order; the BatchNorm sums are fp64
    atomics, whose arrival order varies -- fp64 sums of these bf16-valued terms come out identical in practice
    (the terms would have to span ~20 binades to round differently), which this test checks; it is not a
    guarantee of the arithmetic."""
    from fedmi.engine.cnn_native import CNNNativeTrainer

    nb = 64
    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=128, n_test=64, seed=0)
    init = build_model(name).state_dict()
    runs = []
    for _ in range(2):
        tr = CNNNativeTrainer(name, data, gpu_device, TrainerConfig(batch_size=nb, augment=False, use_graph=False),
                              init_state=init)
        for _ in range(2):          # second pass: statistics shifted by the first pass's batch mean
            tr.grads_for_batch(0, nb)
        torch.cuda.synchronize()
        runs.append(({k: p.grad.clone() for k, p in tr.model.named_parameters()},
                     {k: b.clone() for k, b in tr.model.named_buffers()}, tr.train_stats()))
    (ga, ba, sa), (gb, bb, sb) = runs
    bad = [k for k in ga if not torch.equal(ga[k], gb[k])]
    assert not bad, f"{len(bad)} / {len(ga)} gradients differ between identical runs: {bad[:5]}"
    badb = [k for k in ba if not torch.equal(ba[k], bb[k])]
    assert not badb, badb[:5]
    assert sa.correct == sb.correct and sa.count == sb.count


@pytest.mark.parametrize("name", ["ResNet18", "MobileNet", "GoogLeNet", "PreActResNet18"])
def test_deferred_wgrad_reductions_are_bit_identical(gpu_device, name, monkeypatch):
    """The deferred WGRAD reductions (one wgrad_reduce_multi launch after the backward pass, every conv's
    partials in a buffer of its own) give bit-identical weight gradients to the per-conv reduce launches
    (FEDMI_WRED_DEFER=0), at the full batch and at a partial last batch."""
    from fedmi.engine.cnn_native import CNNNativeTrainer

    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=256, n_test=64, seed=0)
    init = build_model(name).state_dict()
    runs = []
    for defer, cap_mb in (("1", "inf"), ("1", "8"), ("0", "inf")):   # all deferred (default) / a size split / none
        monkeypatch.setenv("FEDMI_WRED_DEFER", defer)
        monkeypatch.setenv("FEDMI_WRED_DEFER_MB", cap_mb)
        tr = CNNNativeTrainer(name, data, gpu_device, TrainerConfig(batch_size=128, augment=False, use_graph=False),
                              init_state=init)
        assert bool(tr._wpart) == (defer == "1")
        grads = []
        for start, nb in ((0, 128), (128, 80)):
            tr.grads_for_batch(start, nb)
            torch.cuda.synchronize()
            grads.append({k: p.grad.clone() for k, p in tr.model.named_parameters()})
        runs.append(grads)
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            bad = [k for k in a if not torch.equal(a[k], b[k])]
            assert not bad, f"{len(bad)} / {len(a)} gradients differ: {bad[:5]}"


# Bounds from profiles/r4_tests/grad_cosines.jsonl (tools/diag_grad_cosines.py, one batch of 64 at random init).
# A tensor is WELL-CONDITIONED when PyTorch's own autocast-bf16 gradient keeps cos >= 0.9 to fp32: there the
# native engine must stay within 0.05 of torch-bf16 (ResNet-18: all 62 tensors, worst gap -0.022).  On the
# rest -- 163 of MobileNetV2's 173 tensors, whose deep BN stack makes every bf16 model's gradient direction
# chaotic at init (torch-bf16 vs fp32 mean cos 0.48 there, min -0.25) -- a single tensor's cosine is noise
# (two runs of the diagnostic put the worst gap on different tensors, -0.29 and -0.44), so the bound is on
# the group: native's mean within 0.05 of torch-bf16's, and no tensor more than 0.6 below it.
# STRUCTURAL ZEROS are left out of every cosine: a BN bias whose output reaches the loss only through train-mode
# BNs (MobileNetV2's every bn3.bias / shortcut.1.bias) has an exactly-zero gradient -- fp64 RMS ~1e-18 against a
# median tensor's 1.8e-3, fp32 1e-10..1e-7 of pure rounding -- so its cosine to fp32 is a coin flip for any
# engine (native -0.69 vs torch-bf16 0.12 on layers.0.bn3.bias in one run).  They are found with an fp64 CPU
# reference; instead of a cosine, the native rounding residue on them (group RMS) must stay within
# STRUCT_ZERO_VS_BF16 of torch-bf16's. (measured: 21 tensors, native 1.6e-4 vs torch-bf16 2.4e-4 vs fp32 1.1e-7).
WELL_COND, WELL_MARGIN, ILL_MEAN_MARGIN, ILL_MAX_GAP = 0.9, 0.05, 0.05, 0.6
STRUCT_ZERO_REL, STRUCT_ZERO_VS_BF16 = 1e-9, 2.0


@pytest.mark.parametrize("name", ["ResNet18", "MobileNetV2"])
def test_native_gradients_track_torch_bf16(gpu_device, name):
    """cos(native grad, fp32 grad) against cos(torch autocast-bf16 grad, fp32 grad): per tensor within 0.05
    where torch-bf16 is well-conditioned, as a group mean elsewhere (see WELL_COND); the mean over all tensors
    within 0.03 of torch-bf16's; the classifier and the last BN at >= 0.99; the loss within 0.5 % of the
    emulated-kernel engine's (same schedule and bf16 buffers, tests/emulate.py)."""
    from fedmi.engine.cnn_native import CNNNativeTrainer
    from emulate import emulated

    nb = 64
    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=128, n_test=64, seed=0)
    torch.manual_seed(0)
    init = build_model(name).state_dict()
    grads, stats = {}, {}
    for kind in ("native", "emulated"):
        cfg = TrainerConfig(batch_size=nb, augment=False, use_graph=False)
        if kind == "native":
            tr = CNNNativeTrainer(name, data, gpu_device, cfg, init_state=init)
            tr.grads_for_batch(0, nb)
        else:
            with emulated():
                tr = CNNNativeTrainer(name, data, gpu_device, cfg, init_state=init)
                tr.grads_for_batch(0, nb)
        torch.cuda.synchronize()
        grads[kind] = {k: p.grad.detach().float().clone() for k, p in tr.model.named_parameters()}
        stats[kind] = tr.train_stats()
    x = augment_normalize(data.train.x[:nb], None, 0, 0)
    y = data.train.y[:nb].long()
    for kind in ("fp32", "bf16"):
        ref = build_model(name).to(gpu_device)
        ref.load_state_dict(init)
        ref.train()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=kind == "bf16"):
            loss = F.cross_entropy(ref(x), y)
        loss.backward()
        grads[kind] = {k: p.grad.detach().float().clone() for k, p in ref.named_parameters()}
    ref64 = build_model(name).double()
    ref64.load_state_dict(init)
    ref64.train()
    F.cross_entropy(ref64(x.double().cpu()), y.cpu()).backward()
    rms64 = {k: p.grad.pow(2).mean().sqrt().item() for k, p in ref64.named_parameters()}
    med = sorted(rms64.values())[len(rms64) // 2]
    zero = [k for k in rms64 if rms64[k] < STRUCT_ZERO_REL * med]
    assert len(zero) <= (0 if name == "ResNet18" else 40), zero
    if zero:
        res = {kind: (sum(grads[kind][k].pow(2).mean().item() for k in zero) / len(zero)) ** 0.5
               for kind in ("native", "bf16", "fp32")}
        print(f"structural zeros: {len(zero)} tensors, residue RMS {res} (median tensor RMS {med:.3e})")
        assert res["native"] < STRUCT_ZERO_VS_BF16 * res["bf16"], res
    assert abs(stats["native"].loss - stats["emulated"].loss) < 5e-3 * stats["emulated"].loss
    names = [k for k in grads["native"] if k not in zero]
    cn = {k: _cos(grads["native"][k], grads["fp32"][k]) for k in names}
    cb = {k: _cos(grads["bf16"][k], grads["fp32"][k]) for k in names}
    well = [k for k in names if cb[k] >= WELL_COND]
    ill = [k for k in names if cb[k] < WELL_COND]
    bad = {k: (round(cn[k], 3), round(cb[k], 3)) for k in well if cn[k] < cb[k] - WELL_MARGIN}
    assert not bad, bad
    if ill:
        assert sum(cn[k] for k in ill) / len(ill) > sum(cb[k] for k in ill) / len(ill) - ILL_MEAN_MARGIN
        bad = {k: (round(cn[k], 3), round(cb[k], 3)) for k in ill if cn[k] < cb[k] - ILL_MAX_GAP}
        assert not bad, bad
    assert sum(cn.values()) / len(names) > sum(cb.values()) / len(names) - 0.03
    tail = ["linear.weight", "linear.bias"] + (["layer4.1.bn2.weight", "layer4.1.bn2.bias"] if name == "ResNet18"
                                               else ["bn2.weight", "bn2.bias"])
    for k in tail:
        assert cn[k] > 0.99 and _cos(grads["native"][k], grads["emulated"][k]) > 0.99, (k, cn[k])


@pytest.mark.parametrize("name", ["ResNet18", "MobileNet", "VGG11", "PreActResNet18", "GoogLeNet"])
def test_native_trains_like_torch_engine(gpu_device, name):
    from fedmi.engine.cnn_native import CNNNativeTrainer
    from fedmi.engine.torch_engine import TorchTrainer

    data = make_dataset("synthetic-cifar10-easy", device=gpu_device, n_train=2560, n_test=1000, seed=0)
    cfg = TrainerConfig(batch_size=128, lr=0.02, seed=7, use_graph=True)
    init = build_model(name).state_dict()
    res = {}
    for kind in ("native", "torch"):
        tr = (CNNNativeTrainer(name, data, gpu_device, cfg, init_state=init) if kind == "native"
              else TorchTrainer(name, data, gpu_device, cfg, init_state=init))
        tr.set_schedule(*contiguous_schedule(len(data.train), 128))
        losses = []
        for _ in range(4):
            tr.train_epoch()
            losses.append(tr.train_stats().loss)
        tr.evaluate()
        res[kind] = (losses, tr.eval_stats())
    (ln, en), (lt, et) = res["native"], res["torch"]
    assert ln[-1] < 0.7 * ln[0], ln
    assert en.count == et.count == 1000
    assert en.acc > 60.0 and en.acc > et.acc - 10.0, (en.acc, et.acc, ln, lt)


def test_graph_replay_equals_eager(gpu_device):
    """SGD steps from one init: captured-graph replay and eager launches give BIT-IDENTICAL models
    (fp64 BN accumulation, fixed-order reductions, the capture's warm-up step fully undone)."""
    from fedmi.engine.cnn_native import CNNNativeTrainer

    data = make_dataset("synthetic-cifar10-easy", device=gpu_device, n_train=256, n_test=500, seed=0)
    init = build_model("ResNet18").state_dict()
    runs = []
    for graph in (False, False, True):
        tr = CNNNativeTrainer("ResNet18", data, gpu_device,
                              TrainerConfig(batch_size=128, lr=0.05, use_graph=graph, seed=3), init_state=init)
        tr.set_schedule([0, 128], [128, 128])
        before = tr.float_state().clone()
        tr.train_epoch()
        runs.append((tr.float_state().clone(), tr.train_stats(), before))
    (e1, s1, b0), (e2, s2, _), (g, sg, _) = runs
    assert not torch.equal(e1, b0)
    assert torch.equal(e1, e2)
    assert torch.equal(e1, g)
    assert s1.count == sg.count == 256 and s1.correct == sg.correct
