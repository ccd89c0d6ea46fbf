"""The native aten backend (fedmi/ops/native_mode.py, csrc/kernels/zoo_ops.hip) vs PyTorch fp32.

Per op: forward outputs and autograd gradients of each native implementation against the same
op in fp32 PyTorch (operands rounded to bf16 first, so the comparison isolates accumulation
error).  Per family: a training step of every zoo family without a whole-network engine runs
under the mode in strict mode (any aten op without a native kernel raises) and tracks the fp32
engine's loss; the HIP-graph replay of the step matches eager execution.
"""
import math

import pytest
import torch
import torch.nn.functional as F
from torch import nn

from fedmi.engine.base import TrainerConfig
from fedmi.engine.data import contiguous_schedule, make_dataset
from fedmi.models import build_model

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6))


def _mode(**kw):
    from fedmi.ops.native_mode import NativeMode

    return NativeMode(strict=True, **kw)


def _bf(t):
    return t.bfloat16().float()


def _run_pair(gpu_device, make, x_shape, seed=0, cl=True, tol=1e-2, gy_dtype=torch.bfloat16):
    """ref: fp32 module on fp32 input; nat: same weights, bf16 channels-last input, under the mode."""
    torch.manual_seed(seed)
    ref = make().to(gpu_device)
    nat = make().to(gpu_device)
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(_bf(p))
    nat.load_state_dict(ref.state_dict())
    x = _bf(torch.randn(*x_shape, device=gpu_device))
    xr = x.clone().requires_grad_(True)
    xn = x.clone()
    if cl and xn.dim() == 4:
        xn = xn.contiguous(memory_format=torch.channels_last)
    xn = xn.to(torch.bfloat16).requires_grad_(True)
    yr = ref(xr)
    mode = _mode()
    with mode:
        yn = nat(xn)
    gy = _bf(torch.randn_like(yr))
    yr.backward(gy)
    with mode:
        yn.backward(gy.to(yn.dtype))
    torch.cuda.synchronize()
    assert not mode.fallbacks, dict(mode.fallbacks)
    assert yn.shape == yr.shape
    assert _rel(yn, yr) < tol, ("y", _rel(yn, yr))
    assert _rel(xn.grad, xr.grad) < tol, ("dx", _rel(xn.grad, xr.grad))
    for (n, pr), pn in zip(ref.named_parameters(), nat.parameters()):
        assert pn.grad is not None, n
        assert _rel(pn.grad, pr.grad) < tol, (n, _rel(pn.grad, pr.grad))
    for (n, br), bn in zip(ref.named_buffers(), nat.buffers()):
        if br.is_floating_point():
            assert _rel(bn, br) < 1e-3, (n, _rel(bn, br))
    return mode


# (N, H, C, O, k, stride, pad, groups, bias): MFMA dense (DenseNet 1x1 C % 64 != 0, strided 3x3 / 1x1
# shortcuts, 5x5 / 7x7), depthwise, grouped MFMA (ResNeXt 2x64d), VALU grouped (ResNeXt 32x4d, DPN,
# RegNet, ShuffleNet g3 widths), the 3-channel stem, a biased conv
CONVS = [(8, 16, 24, 48, 1, 1, 0, 1, False), (8, 16, 48, 16, 3, 1, 1, 1, False), (4, 16, 64, 128, 3, 2, 1, 1, False),
         (4, 16, 64, 128, 1, 2, 0, 1, True), (2, 16, 32, 64, 5, 1, 2, 1, False), (2, 16, 16, 32, 7, 2, 3, 1, False),
         (8, 16, 32, 32, 3, 1, 1, 32, False), (4, 16, 64, 64, 5, 2, 2, 64, False), (4, 16, 128, 128, 3, 1, 1, 2, False),
         (4, 8, 128, 128, 3, 2, 1, 32, False), (4, 8, 96, 96, 3, 1, 1, 3, False), (4, 8, 60, 60, 1, 1, 0, 3, False),
         (4, 16, 3, 64, 3, 1, 1, 1, False), (4, 16, 58, 58, 1, 1, 0, 1, True),
         (4, 8, 160, 160, 3, 2, 1, 10, False), (4, 4, 384, 384, 3, 1, 1, 24, False),   # RegNetY group width 16
         (4, 16, 64, 64, 3, 1, 1, 4, False), (4, 16, 200, 200, 1, 1, 0, 2, False),    # 4 x 16 groups, ShuffleNet
         (4, 8, 96, 96, 3, 1, 1, 32, False), (4, 8, 192, 192, 3, 2, 1, 32, False),     # DPN: 3- / 6- / 12-channel
         (2, 8, 384, 384, 3, 1, 1, 32, False),                                          # groups: block-diagonal MFMA
         (4, 8, 60, 60, 3, 1, 1, 12, False),                                            # off-grid widths: direct gconv
         (4, 16, 44, 44, 7, 1, 3, 44, False), (4, 16, 44, 44, 3, 2, 1, 44, False)]     # PNASNetA depthwise, padded


@pytest.mark.parametrize("shape", CONVS, ids=[str(s) for s in CONVS])
def test_conv_fwd_bwd(gpu_device, shape):
    N, H, C, O, k, st, pad, g, bias = shape
    _run_pair(gpu_device, lambda: nn.Conv2d(C, O, k, st, pad, groups=g, bias=bias), (N, C, H, H))


def test_batchnorm_train_eval(gpu_device):
    def make():
        return nn.Sequential(nn.BatchNorm2d(48), nn.ReLU())
    mode = _run_pair(gpu_device, make, (16, 48, 8, 8))
    assert (mode.native_ops["aten.native_batch_norm.default"] + mode.native_ops["aten.miopen_batch_norm.default"]) == 1
    # eval: running statistics path
    torch.manual_seed(3)
    ref = nn.BatchNorm2d(16).to(gpu_device)
    with torch.no_grad():
        ref.running_mean.uniform_(-1, 1)
        ref.running_var.uniform_(0.5, 2)
        ref.weight.uniform_(0.5, 1.5)
    ref.eval()
    x = _bf(torch.randn(8, 16, 6, 6, device=gpu_device))
    with _mode():
        yn = ref(x.contiguous(memory_format=torch.channels_last).bfloat16())
    assert _rel(yn, ref(x)) < 1e-2


def test_batchnorm_large_mean(gpu_device):
    """Moments are taken about the running mean: a channel whose mean dwarfs its spread keeps its
    variance (E[x^2] - E[x]^2 in fp32 would cancel)."""
    bn = nn.BatchNorm2d(8).to(gpu_device)
    with torch.no_grad():
        bn.running_mean.fill_(100.0)
    x = 100.0 + torch.randn(32, 8, 8, 8, device=gpu_device)
    ref = nn.BatchNorm2d(8).to(gpu_device)
    with torch.no_grad():
        ref.running_mean.fill_(100.0)
    yr = ref(x)
    with _mode():
        yn = bn(x)
    assert _rel(yn, yr) < 1e-3
    assert _rel(bn.running_var, ref.running_var) < 1e-3


class _SE(nn.Module):
    """SE gate + residual add + concat + slice: the mul / sigmoid / mean / cat / slice_backward ops."""

    def __init__(self, c=32):
        super().__init__()
        self.fc1 = nn.Conv2d(c, c // 4, 1)
        self.fc2 = nn.Conv2d(c // 4, c, 1)

    def forward(self, x):
        w = F.adaptive_avg_pool2d(x.float(), 1).to(x.dtype)
        w = torch.sigmoid(self.fc2(F.relu(self.fc1(w))))
        y = x * w + x
        z = torch.cat([y, x[:, : x.shape[1] // 2]], 1)
        return z[:, 8:] * 0.5


def test_se_concat_slice(gpu_device):
    _run_pair(gpu_device, _SE, (8, 32, 8, 8))


@pytest.mark.parametrize("C", [8, 12, 36, 7, 64])
def test_elementwise_and_reductions_layouts(gpu_device, C):
    """Vector (8 / 4 wide) and scalar launches: channel slices at odd offsets, broadcast operands,
    fp32 / bf16 mixes, channels-last row reductions and generic reductions, against fp32 torch."""
    torch.manual_seed(C)
    big = _bf(torch.randn(4, C + 5, 6, 7, device=gpu_device)).contiguous(memory_format=torch.channels_last)
    xs = big[:, 3:3 + C]                                   # channel slice: unaligned base
    xb = big.bfloat16()[:, 3:3 + C]
    b = torch.randn(C, device=gpu_device)
    mode = _mode()
    with mode:
        y = xb * b.view(1, C, 1, 1) + xb
        z = torch.relu(y)
        s = z.sum((0, 2, 3))
        m = z.float().mean((2, 3), keepdim=True)
        cl = z.contiguous(memory_format=torch.channels_last)
        sc = cl.sum((0, 2, 3))
        w = xs * 0.5 + 1.0
    ref_y = xs * b.view(1, C, 1, 1) + xs
    ref_z = torch.relu(ref_y)
    assert not mode.fallbacks
    assert _rel(y, ref_y) < 1e-2 and _rel(z, ref_z) < 1e-2
    assert _rel(s, ref_z.sum((0, 2, 3))) < 1e-2 and _rel(sc, ref_z.sum((0, 2, 3))) < 1e-2
    assert _rel(m, ref_z.mean((2, 3), keepdim=True)) < 1e-2
    assert torch.allclose(w, xs * 0.5 + 1.0)


@pytest.mark.parametrize("pool", ["max3s2p1", "max2", "avg2", "avg3s1p1", "avg3s2p1_ceil_nopad", "avg4"])
def test_pools(gpu_device, pool):
    mk = {"max3s2p1": lambda: nn.MaxPool2d(3, 2, 1), "max2": lambda: nn.MaxPool2d(2),
          "avg2": lambda: nn.AvgPool2d(2), "avg3s1p1": lambda: nn.AvgPool2d(3, 1, 1),
          "avg3s2p1_ceil_nopad": lambda: nn.AvgPool2d(3, 2, 1, ceil_mode=True, count_include_pad=False),
          "avg4": lambda: nn.AvgPool2d(4)}[pool]
    _run_pair(gpu_device, mk, (4, 16, 9, 9) if "ceil" in pool else (4, 16, 8, 8))


def test_linear_cross_entropy(gpu_device):
    torch.manual_seed(0)
    lin = nn.Linear(64, 10).to(gpu_device)
    ref = nn.Linear(64, 10).to(gpu_device)
    ref.load_state_dict(lin.state_dict())
    x = _bf(torch.randn(32, 64, device=gpu_device))
    y = torch.randint(0, 10, (32,), device=gpu_device)
    xr = x.clone().requires_grad_(True)
    lr_ = F.cross_entropy(ref(xr), y)
    lr_.backward()
    xn = x.bfloat16().requires_grad_(True)
    mode = _mode()
    with mode:
        ln = F.cross_entropy(lin(xn), y)
        ln.backward()
    assert not mode.fallbacks
    assert abs(float(ln) - float(lr_)) < 1e-3 * max(1.0, abs(float(lr_)))
    assert _rel(xn.grad, xr.grad) < 1e-2
    assert _rel(lin.weight.grad, ref.weight.grad) < 1e-3
    assert _rel(lin.bias.grad, ref.bias.grad) < 1e-3


@pytest.mark.parametrize("M,K,N", [(128, 1024, 10), (10, 128, 1024), (128, 10, 1024), (77, 300, 65), (1, 33, 1)])
def test_bf16_gemm_mfma(gpu_device, M, K, N):
    """bf16 mm / addmm (the MFMA kernel) on contiguous and transposed operands vs fp32 matmul of the same
    bf16 values: the shapes of a classifier's forward, weight gradient and input gradient plus ragged ones."""
    torch.manual_seed(M * 7 + K + N)
    a = torch.randn(M, K, device=gpu_device).bfloat16()
    b = torch.randn(K, N, device=gpu_device).bfloat16()
    bias = torch.randn(N, device=gpu_device).bfloat16()
    mode = _mode()
    ref = a.float() @ b.float()
    with mode:
        y0 = torch.mm(a, b)
        y1 = torch.mm(a.t().contiguous().t(), b.t().contiguous().t())
        y2 = torch.addmm(bias, a, b, beta=0.5, alpha=2.0)
    torch.cuda.synchronize()
    assert not mode.fallbacks and y0.dtype == torch.bfloat16
    scale = float(ref.abs().max()) + 1e-6
    assert float((y0.float() - ref).abs().max()) / scale < 1e-2
    assert torch.equal(y0, y1)
    ref2 = 2.0 * ref + 0.5 * bias.float()
    assert float((y2.float() - ref2).abs().max()) / (float(ref2.abs().max()) + 1e-6) < 1e-2


def test_ce_stats(gpu_device):
    from fedmi.ops.native_mode import ce_stats_

    torch.manual_seed(0)
    logits = torch.randn(300, 10, device=gpu_device)
    y = torch.randint(0, 10, (300,), device=gpu_device)
    st = torch.zeros(3, device=gpu_device)
    ce_stats_(logits, y, st)
    ce_stats_(logits.bfloat16(), y, st)
    ref_l = F.cross_entropy(logits, y, reduction="sum") + F.cross_entropy(logits.bfloat16().float(), y, reduction="sum")
    ref_c = (logits.argmax(1) == y).sum() + (logits.bfloat16().float().argmax(1) == y).sum()
    assert abs(float(st[0]) - float(ref_l)) < 1e-3 * float(ref_l)
    assert int(st[1]) == int(ref_c) and int(st[2]) == 600


def test_dropout_and_drop_connect(gpu_device):
    x = torch.ones(64, 256, device=gpu_device, requires_grad=True)
    mode = _mode(seed=5)
    with mode:
        y = F.dropout(x, p=0.25, training=True)
        y.sum().backward()
        m = torch.empty(4096, 1, 1, 1, device=gpu_device).bernoulli_(0.8)
        m2 = torch.empty(4096, 1, 1, 1, device=gpu_device).bernoulli_(0.8)
    torch.cuda.synchronize()
    kept = (y != 0).float().mean().item()
    assert abs(kept - 0.75) < 0.02
    assert torch.allclose(y[y != 0], torch.full_like(y[y != 0], 1 / 0.75))
    assert torch.equal(x.grad, (y != 0).float() / 0.75)      # backward reuses the forward mask
    assert abs(m.mean().item() - 0.8) < 0.03
    assert not torch.equal(m, m2)                             # the device counter advanced
    assert not mode.fallbacks


HYBRID = ["densenet_cifar", "ResNeXt29_2x64d", "ResNeXt29_32x4d", "DPN26", "ShuffleNetG2", "ShuffleNetG3",
          "ShuffleNetV2", "SENet18", "EfficientNetB0", "RegNetX_200MF", "RegNetY_400MF", "PNASNetA", "PNASNetB",
          "DLA", "SimpleDLA", "MLP"]


@pytest.mark.parametrize("name", HYBRID)
def test_family_step_native_only(gpu_device, name):
    """One SGD step of each family under the strict mode: no ATen compute op, loss matches fp32."""
    from fedmi.engine import build_trainer
    from fedmi.engine.torch_engine import TorchTrainer

    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=256, n_test=64, seed=0)
    cfg = TrainerConfig(batch_size=64, lr=0.02, seed=7, augment=False)
    kw = {"in_features": 3 * 32 * 32} if name == "MLP" else {}
    init = build_model(name, **kw).state_dict()
    tr = build_trainer(name, data, gpu_device, cfg, init_state=init)
    assert isinstance(tr, TorchTrainer) and tr.hybrid and tr.mode is not None
    tr.mode.strict = True
    ref = TorchTrainer(name, data, gpu_device, cfg, init_state=init, model_kwargs=kw)
    losses = {}
    for kind, t in (("native", tr), ("fp32", ref)):
        t.set_schedule([0, 64], [64, 64])
        t.train_epoch()
        losses[kind] = t.train_stats().loss
        t.evaluate()
        assert t.eval_stats().count == 64
    assert not tr.mode.fallbacks, dict(tr.mode.fallbacks)
    assert math.isfinite(losses["native"])
    assert abs(losses["native"] - losses["fp32"]) < 0.05 * losses["fp32"] + 0.02, losses


# Against the deterministic fp32 reference (conftest.deterministic_reference), over 3 seeds (init, augmentation and
# dropout streams): the gate is the MEAN final-epoch loss against the fp32 engine's mean, within twice the fp32
# engine's own seed spread (tests/helpers.seed_band) -- a single 3-epoch trajectory moved with every rounding change
#  and vetoed bit-different but kernel-test-clean wins.  Per seed only sanity is asserted (finite,
# learning).  RegNetY_400MF stays at lr 0.005: at 0.02 its first epoch diverges on BOTH engines even with a
# reproducible reference (epoch losses native 6.54 / 3.47 / 2.42 vs fp32 8.13 / 4.12 / 2.46, round-5 GPU run).
# DPN26 likewise at 0.005: at 0.02 one of three seeds still sits in its loss-8 transient at epoch 3 on EITHER
# engine, depending on last-bit rounding (fp32 seed 8: 2.79 / 4.51 / 2.98 in three runs; native 3.16 with the
# generic narrow-channel forward, 7.43 with conv_tap<GEN>) -- that measures the transient, not the engine.
FAMILY_SEEDS = (7, 8, 9)


@pytest.mark.parametrize("name,lr", [("densenet_cifar", 0.02), ("SENet18", 0.02), ("DPN26", 0.005),
                                     ("ResNeXt29_2x64d", 0.02), ("EfficientNetB0", 0.02), ("RegNetY_400MF", 0.005)])
def test_family_trains_like_fp32(gpu_device, deterministic_reference, name, lr):
    """Three short epochs per seed, graph-replayed: the seed-mean trajectory tracks the fp32 engine (round 1's
    hybrid EfficientNet / RegNetY went NaN under replay)."""
    from fedmi.engine import build_trainer
    from fedmi.engine.torch_engine import TorchTrainer
    from helpers import seed_band

    data = make_dataset("synthetic-cifar10-easy", device=gpu_device, n_train=1280, n_test=500, seed=0)
    final = {"native": [], "fp32": []}
    first = {"native": [], "fp32": []}
    for seed in FAMILY_SEEDS:
        cfg = TrainerConfig(batch_size=128, lr=lr, seed=seed)
        torch.manual_seed(seed)
        init = build_model(name).state_dict()
        for kind in ("native", "fp32"):
            # the same RNG stream for both engines (EfficientNet's drop-connect / dropout masks)
            torch.manual_seed(1234 + seed)
            tr = (build_trainer(name, data, gpu_device, cfg, init_state=init) if kind == "native"
                  else TorchTrainer(name, data, gpu_device, cfg, init_state=init))
            if kind == "native":
                assert tr.use_graph
            tr.set_schedule(*contiguous_schedule(len(data.train), 128))
            losses = []
            for _ in range(3):
                tr.train_epoch()
                losses.append(tr.train_stats().loss)
            tr.evaluate()
            ev = tr.eval_stats()
            assert all(math.isfinite(v) for v in losses), (kind, seed, losses)
            assert ev.count == 500 and ev.loss == ev.loss
            if kind == "native":
                assert tr._graph is not None and not tr.mode.fallbacks
            final[kind].append(losses[-1])
            first[kind].append(losses[0])
    # learning on the seed mean (one seed of the deep nets can still sit in its loss-8 transient at epoch 3 --
    # in either engine)
    assert sum(final["native"]) < sum(first["native"]), (first, final)
    # floor: bf16 vs fp32 on a 30-step schedule -- a quarter of the fp32 mean loss plus 0.1 (a broken backward sits at
    # ~2.3 or diverges: far outside); otherwise three fp32 seed deviations
    mf = sum(final["fp32"]) / len(final["fp32"])
    _, _, info = seed_band(final["native"], final["fp32"], floor=0.1 + 0.25 * mf, k=3.0)
    print(name, info)


def test_graph_replay_matches_eager(gpu_device):
    """Replaying the captured step gives the eager launch sequence's trajectory: every reduction of the
    backend is fixed-order, so graph replay and eager execution of the same steps are bit-identical."""
    from fedmi.engine import build_trainer

    data = make_dataset("synthetic-cifar10-easy", device=gpu_device, n_train=1280, n_test=64, seed=0)
    cfg = TrainerConfig(batch_size=128, lr=0.02, seed=7, augment=False)
    init = build_model("SimpleDLA").state_dict()
    out = {}
    for graph in (False, True):
        tr = build_trainer("SimpleDLA", data, gpu_device, cfg, init_state=init)
        tr.use_graph = graph
        tr.set_schedule(*contiguous_schedule(1280, 128))
        losses = []
        for _ in range(3):
            tr.train_epoch()
            losses.append(tr.train_stats().loss)
        out[graph] = losses
        assert (tr._graph is not None) == graph
    (le, lg) = out[False], out[True]
    assert lg[-1] < lg[0] and le[-1] < le[0], out
    assert lg == le, out


# DPN26: paired slice gradients summed as copies; SENet18: SE-gate multiply + sum as one dot reduction
@pytest.mark.parametrize("name", ["densenet_cifar", "ResNeXt29_2x64d", "DLA", "DPN26", "SENet18"])
def test_bn_relu_fusion_is_exact(gpu_device, name):
    """BN -> [residual add ->] ReLU (one pass) and ReLU-backward -> BN-backward (masked sums and apply)
    fusion: relu(bf16(BN(x))) == bf16(relu(BN(x))), the fused add rounds the BN output to bf16 where the
    unfused pair stores it, and the mask is exact, so a training step with the fusion gives BIT-IDENTICAL
    weights to the unfused step (eager, same init and batch)."""
    from fedmi.engine import build_trainer

    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=128, n_test=64, seed=0)
    cfg = TrainerConfig(batch_size=64, lr=0.02, seed=7, augment=False, use_graph=False)
    init = build_model(name).state_dict()
    res = {}
    for fuse in (False, True):
        tr = build_trainer(name, data, gpu_device, cfg, init_state=init)
        tr.use_graph = False
        tr.mode.fuse = fuse
        tr.set_schedule([0, 64], [64, 64])
        tr.train_epoch()
        torch.cuda.synchronize()
        res[fuse] = (tr.float_state().clone(), tr.train_stats(), dict(tr.mode.fused))
    (w0, s0, f0), (w1, s1, f1) = res[False], res[True]
    assert not f0 and f1.get("bn+relu", 0) + f1.get("bn+relu_", 0) > 0 and f1.get("relu_bwd+bn_bwd", 0) > 0, f1
    if name == "ResNeXt29_2x64d":      # identity and projection shortcuts: BN + add + ReLU in one pass
        assert f1.get("bn+add", 0) > 0 and f1.get("bn+add+relu", 0) > 0, f1
    assert torch.equal(w0, w1)
    assert s0.correct == s1.correct and s0.count == s1.count


@pytest.mark.parametrize("name", ["EfficientNetB0", "RegNetY_400MF", "DPN26", "ShuffleNetG2"])
def test_native_backend_is_deterministic(gpu_device, name):
    """Two graph-replayed epochs from the same init give bit-identical weights: every reduction of the
    native aten backend is fixed-order (ordered split partials, no float atomics), so run-to-run
    differences cannot explain a learning gap against fp32."""
    from fedmi.engine import build_trainer

    data = make_dataset("synthetic-cifar10-easy", device=gpu_device, n_train=512, n_test=64, seed=0)
    cfg = TrainerConfig(batch_size=128, lr=0.02, seed=7)
    init = build_model(name).state_dict()
    outs = []
    for _ in range(2):
        tr = build_trainer(name, data, gpu_device, cfg, init_state=init)
        tr.set_schedule(*contiguous_schedule(len(data.train), 128))
        tr.train_epoch()
        torch.cuda.synchronize()
        outs.append((tr.float_state().clone(), tr.train_stats().loss))
    assert torch.equal(outs[0][0], outs[1][0]), float((outs[0][0] - outs[1][0]).abs().max())
    assert outs[0][1] == outs[1][1]


@pytest.mark.parametrize("name", ["densenet_cifar", "RegNetX_200MF", "EfficientNetB0", "ResNeXt29_2x64d"])
def test_deferred_wgrad_reductions_are_bit_identical(gpu_device, name):
    """The aten backend's deferred WGRAD reductions (every WGRAD into a flat-gradient slot keeps its partials; one
    wgrad_reduce_multi launch per 32 at the first read / the mode's flush) give the same weights, bit for bit, as
    reducing each right away (defer_wred off), over graph-replayed steps: same reduce bodies, same split counts."""
    from fedmi.engine import build_trainer

    data = make_dataset("synthetic-cifar10-easy", device=gpu_device, n_train=384, n_test=64, seed=0)
    cfg = TrainerConfig(batch_size=128, lr=0.02, seed=7)
    init = build_model(name).state_dict()
    outs = []
    for defer in (True, False):
        tr = build_trainer(name, data, gpu_device, cfg, init_state=init)
        assert tr.mode is not None, "the zoo family runs on the native aten backend"
        tr.mode.defer_wred = defer
        tr.set_schedule(*contiguous_schedule(len(data.train), 128))
        tr.train_epoch()
        torch.cuda.synchronize()
        outs.append((tr.float_state().clone(), tr.train_stats().loss))
    assert torch.equal(outs[0][0], outs[1][0]), float((outs[0][0] - outs[1][0]).abs().max())
    assert outs[0][1] == outs[1][1]


@pytest.mark.parametrize("C", [24, 36, 48, 252])
@pytest.mark.parametrize("M", [1000, 4096])
def test_bn_rows_bwd_fused_mask_matches_premasked(gpu_device, C, M):
    """The BN-backward row pass with the ReLU mask fused (f = ReLU output) gives BIT-IDENTICAL sums /
    coefficients to the same pass over the pre-masked gradient (what the unfused threshold_backward
    writes) -- the kernel-level half of test_bn_relu_fusion_is_exact."""
    from fedmi import native
    from fedmi.ops.native_mode import _DT

    nat = native.require()
    st = native.stream_handle(gpu_device)
    g = torch.Generator(device="cpu").manual_seed(C * 7 + M)
    mk = lambda *s: torch.randn(*s, generator=g).to(gpu_device)   # noqa: E731
    gy, x = mk(M, C).bfloat16(), mk(M, C).bfloat16()
    f = torch.relu(mk(M, C)).bfloat16()
    gm = torch.where(f > 0, gy, torch.zeros_like(gy))
    mean, invstd, w = mk(C), mk(C).abs() + 0.5, mk(C)
    outs = []
    for a, ff in ((gy, f), (gm, None)):
        part = torch.empty(int(nat.z_reduce_rows_ws_floats(M, C)), dtype=torch.float32, device=gpu_device)
        o = [torch.full((C,), float("nan"), device=gpu_device) for _ in range(5)]
        nat.z_bn_rows_bwd(st, a.data_ptr(), _DT[a.dtype], C, x.data_ptr(), _DT[x.dtype], C,
                          ff.data_ptr() if ff is not None else 0, _DT[f.dtype] if ff is not None else 0, C, 0.0,
                          mean.data_ptr(), invstd.data_ptr(), w.data_ptr(), C, M, part.data_ptr(), part.numel(),
                          *[t.data_ptr() for t in o])
        outs.append(o)
    torch.cuda.synchronize()
    for name, p, q in zip(("k", "b", "c", "dw", "db"), *outs):
        assert torch.equal(p, q), (name, (p - q).abs().max().item())
    ref_db = gm.float().sum(0)
    assert torch.allclose(outs[0][4], ref_db, rtol=1e-4, atol=1e-3)
