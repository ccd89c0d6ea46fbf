"""Numerics of the fused LeNet HIP kernels vs a plain PyTorch fp32 reference.

Every kernel (K1 conv fwd, K2 FC head fwd+CE+bwd, K3 conv bwd, K4 SGD+pack,
the pack kernel and the graph-replayed epoch) is checked against the same op
computed by ``fedmi.models.small.LeNet`` in fp32 with autograd, on the same
augmented inputs (the host twin of the device RNG, fedmi.engine.data.hash3).
The kernels take bf16 MFMA operands with fp32 accumulation, so tolerances are
relative-L2 at the bf16 level.
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


def _run_grad(nat, tr, start, nb, augment, fused=False):
    """K1+K2+K3 via the raw entry points; returns (flat grad, stats).  ``fused``: fc1 inside the tail."""
    L = tr.L
    tr.stats.zero_()
    tr.conv_slab.zero_()
    tr.fc_slab.zero_()
    tr.fc1w_grad.zero_()
    s = _stream()
    nat.lenet_conv_fwd(s, tr.train_set.x.data_ptr(), start, nb, tr.pk.data_ptr(), tr.params.data_ptr(), SEED,
                       tr.round_ctr.data_ptr(), int(augment), tr.act2.data_ptr(), tr.act2T.data_ptr(),
                       L["MAX_TRAIN_BATCH"], tr.pool1.data_ptr(), tr.am1.data_ptr(), tr.am2.data_ptr(),
                       tr.stats[0].data_ptr())
    labels = tr.train_set.y[start:]
    nat.lenet_fc_head(s, tr.act2.data_ptr(), labels.data_ptr(), nb, 1, tr.pk.data_ptr(), tr.params.data_ptr(),
                      0 if fused else tr.h1.data_ptr(), tr.dact2.data_ptr(), tr.dZ1T.data_ptr(),
                      tr.fc_slab.data_ptr(), tr.stats[0].data_ptr())
    nat.lenet_conv_bwd(s, tr.train_set.x.data_ptr(), start, nb, SEED, tr.round_ctr.data_ptr(), int(augment),
                       tr.dact2.data_ptr(), tr.act2T.data_ptr(), tr.dZ1T.data_ptr(), tr.pool1.data_ptr(),
                       tr.am1.data_ptr(), tr.am2.data_ptr(), tr.pk.data_ptr(), tr.conv_slab.data_ptr(),
                       tr.fc1w_grad.data_ptr())
    torch.cuda.synchronize()
    nfc = (nb + L["FC_SPW"] - 1) // L["FC_SPW"]
    g = torch.cat([tr.conv_slab[:nb].sum(0), tr.fc1w_grad, tr.fc_slab[:nfc].sum(0)])
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
    fc1t = pk[off:off + 400 * 128].view(400, 128)
    assert torch.equal(fc1t[:, :120], bf(sd["fc1.weight"].t()))


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


@pytest.mark.parametrize("fused", [False, True], ids=["fc1-kernel", "fc1-in-tail"])
@pytest.mark.parametrize("start,nb,augment", [(0, 128, True), (256, 128, False), (896, 80, True), (128, 33, True)])
def test_step_stagewise_matches_torch(env, start, nb, augment, fused):
    """K2 and K3 vs fp32 torch math fed with the kernels' own saved forward tensors.

    Using K1's act2/pool1/argmax as inputs removes argmax/ReLU flips, so the only
    remaining differences are fp32 summation order: tight tolerances.
    """
    nat, dev, ds, ref, tr = env
    tr.load_state_dict(ref.state_dict())
    tr.round_ctr.zero_()
    g, stats = _run_grad(nat, tr, start, nb, augment, fused=fused)
    L = tr.L
    sd = {k: v.float() for k, v in ref.state_dict().items()}
    W1, W2, W3 = _bf(sd["fc1.weight"]), _bf(sd["fc2.weight"]), _bf(sd["fc3.weight"])
    X = tr.act2[:nb, :400].float()
    y = ds.train.y[start:start + nb].long()
    # ---- K2: FC head, kernel rounding points (H1, H2, dZ3, dZ2, dZ1 in bf16)
    h1 = _bf(torch.relu(X @ W1.t() + sd["fc1.bias"]))
    if not fused:   # the fused tail keeps H1 in LDS
        assert rel(tr.h1[:nb, :120].float(), h1) < 1e-2
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
    assert abs(int(st[1]) - int((z.argmax(1) == y).sum())) <= 1
    dz1k = tr.dZ1T[:120, :nb].float().t()
    assert rel(dz1k, dz1b) < 1e-2
    assert tr.dZ1T[:, nb:].abs().sum().item() == 0                       # K-padding of the fc1 wgrad
    assert rel(tr.dact2[:nb], (dz1k @ W1) * (X > 0)) < 1e-2
    # ---- K3: conv backward from the kernel's d(pool2), pool1 and argmax codes
    C2W, C1W = _bf(sd["conv2.weight"]), _bf(sd["conv1.weight"])
    dxf = tr.dact2[:nb].clone()                                          # d(pool2)  [nb, 400]
    dY2 = _unpool(dxf.view(nb, 16, 5, 5), tr.am2[:nb].view(nb, 16, 5, 5), 5, 5)
    p1 = tr.pool1[:nb].float().view(nb, 6, 14, 14)
    dW2 = torch.nn.grad.conv2d_weight(p1, C2W.shape, _bf(dY2))
    dP1 = torch.nn.grad.conv2d_input(p1.shape, C2W, _bf(dY2)) * (p1 > 0)
    dY1 = _unpool(dP1, tr.am1[:nb].view(nb, 6, 14, 14), 14, 14)
    gidx = np.arange(start, start + nb) if augment else None
    xin = _bf(augment_normalize(ds.train.x[start:start + nb], gidx, SEED, 0))
    dW1 = torch.nn.grad.conv2d_weight(xin, C1W.shape, _bf(dY1))
    exp_conv = {"conv1.weight": dW1, "conv1.bias": dY1.sum((0, 2, 3)),
                "conv2.weight": dW2, "conv2.bias": dY2.sum((0, 2, 3))}
    exp = {**exp_conv, **exp_fc}
    off = 0
    for name, shape in LENET_SPEC:
        k = int(np.prod(shape))
        e = rel(g[off:off + k], exp[name].reshape(-1))
        assert e < 2e-2, f"{name}: rel err {e:.3e}"
        off += k


@pytest.mark.parametrize("start,nb", [(0, 128), (896, 80)])
def test_step_end_to_end_vs_fp32_autograd(env, start, nb):
    """Sanity bound vs the fp32 model (includes the bf16-vs-fp32 model difference)."""
    nat, dev, ds, ref, tr = env
    tr.load_state_dict(ref.state_dict())
    tr.round_ctr.zero_()
    g, stats = _run_grad(nat, tr, start, nb, True)
    gr, out, loss, y = _ref_grad(ref, ds, start, nb, True)
    assert rel(g, gr) < 0.25
    assert abs(float(stats.cpu()[0:1].view(torch.float32)) / nb - loss.item()) < 2e-2 * max(1.0, loss.item())


def test_sgd_kernel_exact(env):
    nat, dev, ds, ref, tr = env
    L = tr.L
    torch.manual_seed(5)
    p0 = torch.randn(L["P_TOTAL"], device=dev)
    m0 = torch.randn(L["P_TOTAL"], device=dev) * 0.1
    tr.params.copy_(p0)
    tr.mom.copy_(m0)
    nb = 100
    nfc = 7
    tr.conv_slab.normal_()
    tr.fc_slab.normal_()
    tr.fc1w_grad.normal_()
    nat.lenet_sgd(_stream(), tr.params.data_ptr(), tr.mom.data_ptr(), tr.pk.data_ptr(), tr.conv_slab.data_ptr(), nb,
                  tr.fc1w_grad.data_ptr(), tr.fc_slab.data_ptr(), nfc, 0.1, 0.9, 5e-4, 0)
    torch.cuda.synchronize()
    g = torch.cat([tr.conv_slab[:nb].double().sum(0), tr.fc1w_grad.double(), tr.fc_slab[:nfc].double().sum(0)])
    d = g + 5e-4 * p0.double()
    b = 0.9 * m0.double() + d
    p = p0.double() - 0.1 * b
    assert torch.allclose(tr.mom.double(), b, rtol=1e-5, atol=1e-5)
    assert torch.allclose(tr.params.double(), p, rtol=1e-5, atol=1e-5)
    # packed images follow the master weights
    pk = tr.pk.float()
    w1 = tr.params[:450].view(6, 3, 5, 5).bfloat16().float()
    w1c = pk[:16 * 128].view(16, 128)
    assert torch.equal(w1c[:6, 0:3], w1[:, :, 0, 0])      # group (r=0, s=0..1), channels 0..2
    assert torch.equal(w1c[:6, 4:7], w1[:, :, 0, 1])
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


@pytest.mark.parametrize("use_graph", [True, False], ids=["graph", "eager"])
def test_fused_bwd_sgd_matches_separate_kernels(env, use_graph):
    """K34 (conv backward + SGD in one launch, producer flags -> SGD workgroups) trains like K3 then K4,
    across steps (flag generations) and rounds (augmentation counter bumped once per round)."""
    nat, dev, ds, ref, tr = env
    starts, sizes = [0, 128, 384, 896], [128, 128, 33, 80]
    res = []
    tr.engine.set_sample_path(False)
    for fuse in (False, True):
        tr.engine.set_fuse_head(True)
        tr.engine.set_fuse_sgd(fuse)
        assert tr.engine.fuse_sgd() == fuse
        tr.load_state_dict(ref.state_dict())
        tr.mom.zero_()
        tr.round_ctr.zero_()
        tr.stats.zero_()
        tr.round_idx = 0
        tr.cfg.use_graph = use_graph
        tr.set_schedule(starts, sizes)
        for _ in range(2):
            tr.train_epoch()
        torch.cuda.synchronize()
        res.append((tr.params.clone(), tr.mom.clone(), tr.train_stats(), int(tr.stats[0][3]),
                    int(tr.round_ctr[0])))
    (p0, m0, s0, e0, r0), (p1, m1, s1, e1, r1) = res
    assert e0 == 0 and e1 == 0, "hand-off timed out"
    assert r0 == r1 == 2
    assert s0.count == s1.count == sum(sizes) and s0.correct == s1.correct
    assert abs(s0.loss_sum - s1.loss_sum) <= 1e-4 * abs(s0.loss_sum)
    assert rel(p1, p0) < 1e-5 and rel(m1, m0) < 1e-5   # only the LDS-atomic order of K3's bias sums differs
    tr.engine.set_fuse_sgd(False)
    tr.engine.set_sample_path(True)


@pytest.mark.parametrize("use_graph", [True, False], ids=["graph", "eager"])
def test_fused_fwd_head_matches_separate_kernels(env, use_graph):
    """K12 (conv stack + FC head in one launch, flag hand-off) trains exactly like K1 then K2b."""
    nat, dev, ds, ref, tr = env
    starts, sizes = [0, 128, 384, 896], [128, 128, 33, 80]      # full and partial batches
    res = []
    tr.engine.set_sample_path(False)
    for fuse in (False, True):
        tr.engine.set_fuse_head(fuse)
        tr.load_state_dict(ref.state_dict())
        tr.mom.zero_()
        tr.round_ctr.zero_()
        tr.round_idx = 0
        tr.cfg.use_graph = use_graph
        tr.set_schedule(starts, sizes)
        tr.train_epoch()
        torch.cuda.synchronize()
        res.append((tr.params.clone(), tr.train_stats(), int(tr.stats[0][3])))
    (p0, s0, e0), (p1, s1, e1) = res
    assert e1 == 0, "K12 hand-off timed out"
    assert s0.count == s1.count == sum(sizes) and s0.correct == s1.correct
    assert abs(s0.loss_sum - s1.loss_sum) <= 1e-4 * abs(s0.loss_sum)
    assert rel(p1, p0) < 1e-5          # only the LDS-atomic order of K3's bias sums differs
    tr.engine.set_fuse_head(True)
    tr.engine.set_sample_path(True)
    tr.cfg.use_graph = True
    tr.load_state_dict(ref.state_dict())
    tr.mom.zero_()


@pytest.mark.parametrize("start,nb", [(0, 128), (896, 80), (128, 33)])
def test_sample_step_gradients_match_head_kernels(env, start, nb):
    """KS1 + KS2 (one workgroup per sample, batched FC-gradient GEMMs) compute the same gradients as
    K1 + K2 + K3 (per-tensor rel. L2 at the bf16 level: the FC GEMVs sum in a different order and a
    bf16 rounding of an intermediate may land one ulp apart), the same loss and accuracy."""
    nat, dev, ds, ref, tr = env
    tr.load_state_dict(ref.state_dict())
    tr.round_ctr.zero_()
    g_head, st_head = _run_grad(nat, tr, start, nb, True, fused=True)
    lr, wd = tr.cfg.lr, tr.cfg.weight_decay
    tr.engine.set_sample_path(True)
    tr.load_state_dict(ref.state_dict())
    tr.mom.zero_()
    tr.stats.zero_()
    p0 = tr.params.clone()
    tr.train_step(start, nb)                    # momentum buffer 0: p = p0 - lr * (g + wd * p0)
    torch.cuda.synchronize()
    g = (p0.double() - tr.params.double()) / lr - wd * p0.double()
    off = 0
    for name, shape in LENET_SPEC:
        k = int(np.prod(shape))
        e = rel(g[off:off + k], g_head[off:off + k])
        assert e < 1e-2, f"{name}: rel err {e:.3e}"
        off += k
    st, sh = tr.stats[0].cpu(), st_head.cpu()
    assert int(st[2]) == nb
    assert abs(int(st[1]) - int(sh[1])) <= 1
    ls, lh = float(st[0:1].view(torch.float32)), float(sh[0:1].view(torch.float32))
    assert abs(ls - lh) < 1e-3 * max(1.0, abs(lh))
    assert rel(tr.mom.double(), g + wd * p0.double()) < 1e-4   # g is recovered from fp32 params
    tr.load_state_dict(ref.state_dict())
    tr.mom.zero_()


@pytest.mark.parametrize("use_graph", [True, False], ids=["graph", "eager"])
def test_sample_path_trains_like_head_path(env, use_graph):
    """Two epochs of full and partial batches: the per-sample path and K12 -> K3 -> K4 stay together."""
    nat, dev, ds, ref, tr = env
    starts, sizes = [0, 128, 384, 896], [128, 128, 33, 80]
    res = []
    for sample in (False, True):
        tr.engine.set_sample_path(sample)
        tr.load_state_dict(ref.state_dict())
        tr.mom.zero_()
        tr.round_ctr.zero_()
        tr.stats.zero_()
        tr.round_idx = 0
        tr.cfg.use_graph = use_graph
        tr.set_schedule(starts, sizes)
        for _ in range(2):
            tr.train_epoch()
        torch.cuda.synchronize()
        res.append((tr.params.clone(), tr.train_stats(), int(tr.round_ctr[0])))
    (p0, s0, r0), (p1, s1, r1) = res
    init = torch.cat([v.detach().reshape(-1).float() for v in ref.state_dict().values()])
    assert r0 == r1 == 2
    assert s0.count == s1.count == sum(sizes) and abs(s0.correct - s1.correct) <= 2
    assert abs(s0.loss_sum - s1.loss_sum) <= 2e-3 * abs(s0.loss_sum)
    assert rel(p1 - init, p0 - init) < 5e-2      # 8 SGD steps of bf16-level differences
    tr.engine.set_sample_path(True)
    tr.cfg.use_graph = True
    tr.load_state_dict(ref.state_dict())
    tr.mom.zero_()
