"""Numerics of the fused LeNet HIP kernels vs a plain PyTorch fp32 reference.

The training step (KS1 lenet_sample_step + KS2 lenet_sgd2), the eval kernels
(lenet_conv_fwd, lenet_fc_eval, lenet_eval_stats), the pack kernel and the
graph-replayed epoch are checked against the same op computed by
``fedmi.models.small.LeNet`` in fp32 (autograd or the explicit backward math),
on the same augmented inputs (the host twin of the device RNG,
fedmi.engine.data.hash3).  The kernels take bf16 MFMA operands with fp32
accumulation, so tolerances are relative-L2 at the bf16 level.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fedmi import native
from fedmi.engine.base import TrainerConfig
from fedmi.engine.data import augment_normalize, make_dataset, strided_schedule
from fedmi.engine.lenet_native import LENET_SPEC, LeNetNativeTrainer
from fedmi.models.small import LeNet

pytestmark = pytest.mark.gpu

SEED = 1234


def rel(a, b):
    a = a.double().flatten()
    b = b.double().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def env(gpu_device):
    nat = native.require()
    dev = gpu_device
    ds = make_dataset("synthetic-cifar10", n_train=1024, n_test=512, device=dev, seed=3)
    torch.manual_seed(0)
    ref = LeNet().to(dev)
    cfg = TrainerConfig(seed=SEED)
    tr = LeNetNativeTrainer(ds, dev, cfg, init_state=ref.state_dict())
    torch.cuda.synchronize()
    return nat, dev, ds, ref, tr


def _stream():
    return native.stream_handle()


def _forward_oracle(nat, tr, start, nb, augment):
    """The eval conv stack (lenet_conv_fwd) in "train" mode over the batch: act2 / pool1 / argmax codes
    (KS1 computes the same forward with the same MFMA order, so its argmaxes are these)."""
    L = tr.L
    dev = tr.params.device
    pool1 = torch.zeros(nb, L["NP1"], dtype=torch.bfloat16, device=dev)
    am1 = torch.zeros(nb, L["NP1"], dtype=torch.uint8, device=dev)
    am2 = torch.zeros(nb, L["F0"], dtype=torch.uint8, device=dev)
    act2T = torch.zeros(L["F0P"], L["MAX_TRAIN_BATCH"], dtype=torch.bfloat16, device=dev)
    nat.lenet_conv_fwd(_stream(), tr.train_set.x.data_ptr(), start, nb, tr.pk.data_ptr(), tr.params.data_ptr(), SEED,
                       tr.round_ctr.data_ptr(), int(augment), tr.act2.data_ptr(), act2T.data_ptr(),
                       L["MAX_TRAIN_BATCH"], pool1.data_ptr(), am1.data_ptr(), am2.data_ptr(), 0)
    torch.cuda.synchronize()
    return tr.act2[:nb, :400].float().clone(), pool1, am1, am2


def _step_grad(tr, start, nb):
    """KS1 + KS2 for one batch from zero momentum; returns (flat grad, stats row).  The gradient is
    recovered from the SGD update: p = p0 - lr * (g + wd * p0)."""
    lr, wd = tr.cfg.lr, tr.cfg.weight_decay
    tr.mom.zero_()
    tr.stats.zero_()
    p0 = tr.params.clone()
    tr.train_step(start, nb)
    torch.cuda.synchronize()
    g = (p0.double() - tr.params.double()) / lr - wd * p0.double()
    assert rel(tr.mom.double(), g + wd * p0.double()) < 1e-4   # momentum buffer = d of the first step
    return g, tr.stats[0].clone()


class _Q(torch.autograd.Function):
    """Round to bf16 where the kernels do (forward operands); identity gradient."""

    @staticmethod
    def forward(ctx, t):
        return t.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g


def _emulated_forward(m, x):
    q = _Q.apply
    h = F.max_pool2d(F.relu(m.conv1(q(x))), 2)
    h = F.max_pool2d(F.relu(m.conv2(q(h))), 2)
    h = q(F.relu(m.fc1(q(torch.flatten(h, 1)))))
    h = q(F.relu(m.fc2(h)))
    return m.fc3(h)


def _ref_grad(ref, ds, start, nb, augment, round_idx=0, emulate_bf16=False):
    x = ds.train.x[start:start + nb]
    gidx = np.arange(start, start + nb) if augment else None
    xin = augment_normalize(x, gidx, SEED, round_idx)
    y = ds.train.y[start:start + nb].long()
    m = ref
    if emulate_bf16:
        m = LeNet().to(xin.device)
        m.load_state_dict({k: v.bfloat16().float() for k, v in ref.state_dict().items()})
    m.zero_grad()
    out = _emulated_forward(m, xin) if emulate_bf16 else m(xin)
    loss = F.cross_entropy(out, y)
    loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    return g, out.detach(), loss.detach(), y


def test_pack_layout(env):
    nat, dev, ds, ref, tr = env
    tr.engine.pack(_stream())
    torch.cuda.synchronize()
    pk = tr.pk.float().cpu()
    sd = {k: v.float().cpu() for k, v in ref.state_dict().items()}
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    w1 = bf(sd["conv1.weight"])
    w1c = pk[0:16 * 128].view(16, 128)
    exp1 = torch.zeros(16, 128)
    for r in range(5):
        for s_ in range(5):
            g, t = r * 3 + s_ // 2, (s_ & 1) * 4
            exp1[:6, g * 8 + t:g * 8 + t + 3] = w1[:, :, r, s_]
    assert torch.equal(w1c, exp1)
    off = 16 * 128
    w2 = bf(sd["conv2.weight"])
    w2c = pk[off:off + 16 * 224].view(16, 224)
    exp2 = torch.zeros(16, 224)
    exp2[:, :200].view(16, 25, 8)[:, :, :6] = w2.permute(0, 2, 3, 1).reshape(16, 25, 6)
    assert torch.equal(w2c, exp2)
    off += 16 * 224
    w2dg = pk[off:off + 16 * 416].view(16, 416)
    exp3 = torch.zeros(16, 416)
    exp3[:6, :400] = w2.permute(1, 2, 3, 0).reshape(6, 400)
    assert torch.equal(w2dg, exp3)
    off += 16 * 416
    fc1 = pk[off:off + 128 * 416].view(128, 416)
    assert torch.equal(fc1[:120, :400], bf(sd["fc1.weight"]))
    assert fc1[120:].abs().sum() == 0 and fc1[:, 400:].abs().sum() == 0
    off += 128 * 416
    fc2 = pk[off:off + 96 * 128].view(96, 128)
    assert torch.equal(fc2[:84, :120], bf(sd["fc2.weight"]))
    off += 96 * 128
    fc2t = pk[off:off + 128 * 96].view(128, 96)
    assert torch.equal(fc2t[:120, :84], bf(sd["fc2.weight"].t()))
    off += 128 * 96
    fc3 = pk[off:off + 16 * 96].view(16, 96)
    assert torch.equal(fc3[:10, :84], bf(sd["fc3.weight"]))
    assert fc3[10:].abs().sum() == 0 and fc3[:, 84:].abs().sum() == 0
    assert off + 16 * 96 == pk.numel()


def test_conv_fwd_matches_torch(env):
    nat, dev, ds, ref, tr = env
    n = 256
    s = _stream()
    nat.lenet_conv_fwd(s, tr.test_set.x.data_ptr(), 0, n, tr.pk.data_ptr(), tr.params.data_ptr(), 0,
                       tr.round_ctr.data_ptr(), 0, tr.act2.data_ptr(), 0, 0, 0, 0, 0, 0)
    torch.cuda.synchronize()
    got = tr.act2[:n, :400].float()
    with torch.no_grad():
        exp = ref.features(augment_normalize(ds.test.x[:n], None, 0, 0))
    assert rel(got, exp) < 2e-2
    assert tr.act2[:n, 400:].abs().sum().item() == 0


def test_eval_matches_torch(env):
    nat, dev, ds, ref, tr = env
    tr.evaluate()
    st = tr.eval_stats()
    with torch.no_grad():
        out = ref(augment_normalize(ds.test.x, None, 0, 0))
        y = ds.test.y.long()
        loss = F.cross_entropy(out, y, reduction="sum").item()
        corr = (out.argmax(1) == y).sum().item()
    assert st.count == len(ds.test.y)
    assert abs(st.loss_sum - loss) / abs(loss) < 1e-2
    assert abs(st.correct - corr) <= 0.02 * len(y) + 2


def _bf(t):
    return t.bfloat16().float()


def _unpool(g, codes, h, w):
    """Route pooled grads [N,C,h,w] to their 2x2 argmax code (0..3) -> [N,C,2h,2w]."""
    n, c = g.shape[:2]
    out = torch.zeros(n, c, h, 2, w, 2, dtype=g.dtype, device=g.device)
    dy, dx = (codes >> 1).long(), (codes & 1).long()
    for a in (0, 1):
        for b in (0, 1):
            out[:, :, :, a, :, b] = torch.where((dy == a) & (dx == b), g, torch.zeros_like(g))
    return out.view(n, c, 2 * h, 2 * w)


@pytest.mark.parametrize("start,nb,augment", [(0, 128, True), (256, 128, False), (896, 80, True), (128, 33, True)])
def test_step_matches_torch_math(env, start, nb, augment):
    """KS1 + KS2 gradients vs fp32 torch math (the explicit backward at the kernels' bf16 rounding
    points: H1, H2, dZ3, dZ2, dZ1, the conv out-grads) fed with the eval conv stack's saved forward
    tensors -- no argmax / ReLU flips, so only fp32 summation order differs: tight per-tensor bounds.
    Also the step's loss sum and correct count."""
    nat, dev, ds, ref, tr = env
    tr.load_state_dict(ref.state_dict())
    tr.round_ctr.zero_()
    if not augment:              # the engine's augmentation flag is fixed at binding time: rebind without it
        tr.cfg.augment = False
        tr.set_train_data(ds.train)
    X, pool1, am1, am2 = _forward_oracle(nat, tr, start, nb, augment)
    try:
        g, stats = _step_grad(tr, start, nb)
    finally:
        if not augment:
            tr.cfg.augment = True
            tr.set_train_data(ds.train)
    sd = {k: v.float() for k, v in ref.state_dict().items()}
    W1, W2, W3 = _bf(sd["fc1.weight"]), _bf(sd["fc2.weight"]), _bf(sd["fc3.weight"])
    y = ds.train.y[start:start + nb].long()
    # ---- FC head at the kernels' rounding points
    h1 = _bf(torch.relu(X @ W1.t() + sd["fc1.bias"]))
    h2 = _bf(torch.relu(h1 @ W2.t() + sd["fc2.bias"]))
    z = h2 @ W3.t() + sd["fc3.bias"]
    dz = (torch.softmax(z, 1) - F.one_hot(y, 10).float()) / nb
    dzb = _bf(dz)
    dz2 = (dzb @ W3) * (h2 > 0)
    dz2b = _bf(dz2)
    dz1 = (dz2b @ W2) * (h1 > 0)
    dz1b = _bf(dz1)
    exp_fc = {
        "fc3.weight": dzb.t() @ h2, "fc3.bias": dz.sum(0),
        "fc2.weight": dz2b.t() @ h1, "fc2.bias": dz2.sum(0),
        "fc1.weight": dz1b.t() @ _bf(X), "fc1.bias": dz1.sum(0),
    }
    loss = F.cross_entropy(z, y, reduction="sum").item()
    st = stats.cpu()
    assert int(st[2]) == nb
    assert abs(float(st[0:1].view(torch.float32)) - loss) < 1e-3 * max(1.0, abs(loss))
    # argmax flips only where the two top logits are within the kernels' rounding noise: H1 / H2 are bf16
    # (an fp32 summation-order difference can move a value across a bf16 rounding boundary, 2^-8 relative)
    top2 = z.topk(2, 1).values
    ties = int(((top2[:, 0] - top2[:, 1]) < 1e-2 * z.abs().amax(1).clamp_min(1e-3)).sum())
    assert abs(int(st[1]) - int((z.argmax(1) == y).sum())) <= ties + 1
    # ---- conv backward from d(pool2) and the saved pool1 / argmax codes
    dX = (dz1b @ W1) * (X > 0)                                            # d(pool2)  [nb, 400]
    C2W, C1W = _bf(sd["conv2.weight"]), _bf(sd["conv1.weight"])
    dY2 = _unpool(dX.view(nb, 16, 5, 5), am2.view(nb, 16, 5, 5), 5, 5)
    p1 = pool1.float().view(nb, 6, 14, 14)
    dW2 = torch.nn.grad.conv2d_weight(p1, C2W.shape, _bf(dY2))
    dP1 = torch.nn.grad.conv2d_input(p1.shape, C2W, _bf(dY2)) * (p1 > 0)
    dY1 = _unpool(dP1, am1.view(nb, 6, 14, 14), 14, 14)
    gidx = np.arange(start, start + nb) if augment else None
    xin = _bf(augment_normalize(ds.train.x[start:start + nb], gidx, SEED, 0))
    dW1 = torch.nn.grad.conv2d_weight(xin, C1W.shape, _bf(dY1))
    exp = {"conv1.weight": dW1, "conv1.bias": dY1.sum((0, 2, 3)),
           "conv2.weight": dW2, "conv2.bias": dY2.sum((0, 2, 3)), **exp_fc}
    off = 0
    for name, shape in LENET_SPEC:
        k = int(np.prod(shape))
        e = rel(g[off:off + k], exp[name].reshape(-1))
        assert e < 2e-2, f"{name}: rel err {e:.3e}"
        off += k
    tr.load_state_dict(ref.state_dict())
    tr.mom.zero_()


@pytest.mark.parametrize("start,nb", [(0, 128), (896, 80)])
def test_step_end_to_end_vs_fp32_autograd(env, start, nb):
    """Sanity bound vs the fp32 model (includes the bf16-vs-fp32 model difference)."""
    nat, dev, ds, ref, tr = env
    tr.load_state_dict(ref.state_dict())
    tr.round_ctr.zero_()
    g, stats = _step_grad(tr, start, nb)
    gr, out, loss, y = _ref_grad(ref, ds, start, nb, True)
    assert rel(g, gr) < 0.25
    assert abs(float(stats.cpu()[0:1].view(torch.float32)) / nb - loss.item()) < 2e-2 * max(1.0, loss.item())
    tr.load_state_dict(ref.state_dict())
    tr.mom.zero_()


def test_step_is_deterministic(env):
    """Two identical steps give bit-identical parameters, momentum and stats (every cross-wave and
    cross-sample sum is fixed-order: the conv1 bias partials of the 7 dgrad waves, the slab combine,
    the FC GEMM tiles, the loss)."""
    nat, dev, ds, ref, tr = env
    res = []
    for _ in range(2):
        tr.load_state_dict(ref.state_dict())
        tr.round_ctr.zero_()
        res.append(_step_grad(tr, 128, 128) + (tr.params.clone(),))
    (g0, s0, p0), (g1, s1, p1) = res
    assert torch.equal(p0, p1) and torch.equal(s0, s1)
    tr.load_state_dict(ref.state_dict())
    tr.mom.zero_()


def test_graph_epoch_matches_eager_and_torch(env):
    nat, dev, ds, ref, tr = env
    starts, sizes = strided_schedule(1024, 128, 0, 2)     # 4 batches
    results = []
    for use_graph in (False, True):
        tr.load_state_dict(ref.state_dict())
        tr.mom.zero_()
        tr.round_ctr.zero_()
        tr.round_idx = 0
        tr.cfg.use_graph = use_graph
        tr.set_schedule(starts, sizes)
        tr.train_epoch()
        torch.cuda.synchronize()
        results.append((tr.params.clone(), tr.train_stats()))
    (pe, se), (pg, sg) = results
    assert rel(pg, pe) < 1e-4
    assert se.count == sg.count == sum(sizes)
    assert int(tr.round_ctr[0]) == 1
    # fp32 torch reference of the same epoch (SGD m=0.9 wd=5e-4, momentum from zero)
    torch.manual_seed(0)
    m = LeNet().to(dev)
    m.load_state_dict(ref.state_dict())
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
    for s, n in zip(starts, sizes):
        x = augment_normalize(ds.train.x[s:s + n], np.arange(s, s + n), SEED, 0)
        opt.zero_grad()
        F.cross_entropy(m(x), ds.train.y[s:s + n].long()).backward()
        opt.step()
    pr = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    p0 = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    assert rel(pg - p0, pr - p0) < 0.25   # bf16 model vs fp32 model over 4 steps


def test_training_converges(env):
    nat, dev, ds, ref, tr = env
    tr.load_state_dict(ref.state_dict())
    tr.mom.zero_()
    tr.cfg.use_graph = True
    tr.set_schedule(*strided_schedule(1024, 128, 0, 1))
    tr.set_schedule([], [])
    tr.set_schedule(*strided_schedule(1024, 128, 0, 1))
    accs = []
    for _ in range(8):
        tr.train_epoch()
        st = tr.train_stats()
        assert st.count == 1024 and 0 <= st.correct <= st.count and 0.0 < st.loss < 10.0, st
        accs.append(st.acc)
    tr.evaluate()
    ev = tr.eval_stats()
    assert ev.count == len(ds.test.y)
    assert ev.acc > 12.0 and accs[-1] > accs[0] + 5.0, (ev, accs)
