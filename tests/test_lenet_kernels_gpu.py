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


def _run_grad(nat, tr, start, nb, augment):
    """K1+K2+K3 via the raw entry points; returns (flat grad, dact2, stats)."""
    L = tr.L
    tr.stats.zero_()
    tr.conv_slab.zero_()
    tr.fc_slab.zero_()
    s = _stream()
    nat.lenet_conv_fwd(s, tr.train_set.x.data_ptr(), start, nb, tr.pk.data_ptr(), tr.params.data_ptr(), SEED,
                       tr.round_ctr.data_ptr(), int(augment), tr.act2.data_ptr(), tr.act2T.data_ptr(),
                       L["MAX_TRAIN_BATCH"], tr.pool1.data_ptr(), tr.am1.data_ptr(), tr.am2.data_ptr())
    labels = tr.train_set.y[start:]
    nat.lenet_fc_head(s, tr.act2.data_ptr(), tr.act2T.data_ptr(), L["MAX_TRAIN_BATCH"], labels.data_ptr(), nb, 1,
                      tr.pk.data_ptr(), tr.params.data_ptr(), tr.dact2.data_ptr(), tr.fc_slab.data_ptr(),
                      tr.stats[0].data_ptr())
    nat.lenet_conv_bwd(s, tr.train_set.x.data_ptr(), start, nb, SEED, tr.round_ctr.data_ptr(), int(augment),
                       tr.dact2.data_ptr(), tr.pool1.data_ptr(), tr.am1.data_ptr(), tr.am2.data_ptr(),
                       tr.pk.data_ptr(), tr.conv_slab.data_ptr())
    torch.cuda.synchronize()
    nfc = (nb + L["FC_SPW"] - 1) // L["FC_SPW"]
    g = torch.cat([tr.conv_slab[:nb].sum(0), tr.fc_slab[:nfc].sum(0)])
    return g, tr.dact2[:nb].clone(), tr.stats[0].clone()


def _ref_grad(ref, ds, start, nb, augment, round_idx=0):
    x = ds.train.x[start:start + nb]
    gidx = np.arange(start, start + nb) if augment else None
    xin = augment_normalize(x, gidx, SEED, round_idx)
    y = ds.train.y[start:start + nb].long()
    ref.zero_grad()
    out = ref(xin)
    loss = F.cross_entropy(out, y)
    loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    return g, out.detach(), loss.detach(), y


def test_pack_layout(env):
    nat, dev, ds, ref, tr = env
    tr.engine.pack(_stream())
    torch.cuda.synchronize()
    pk = tr.pk.float().cpu()
    sd = {k: v.float().cpu() for k, v in ref.state_dict().items()}
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    w1c = pk[0:16 * 96].view(16, 96)
    assert torch.equal(w1c[:6, :75], bf(sd["conv1.weight"].view(6, 75)))
    assert w1c[6:].abs().sum() == 0 and w1c[:, 75:].abs().sum() == 0
    off = 16 * 96
    w2c = pk[off:off + 16 * 160].view(16, 160)
    assert torch.equal(w2c[:, :150], bf(sd["conv2.weight"].view(16, 150)))
    off += 16 * 160
    w2dg = pk[off:off + 16 * 416].view(16, 416)
    exp = sd["conv2.weight"].permute(1, 0, 2, 3).reshape(6, 400)
    assert torch.equal(w2dg[:6, :400], bf(exp))
    off += 16 * 416
    fc1 = pk[off:off + 128 * 416].view(128, 416)
    assert torch.equal(fc1[:120, :400], bf(sd["fc1.weight"]))
    off += 128 * 416
    fc1t = pk[off:off + 400 * 128].view(400, 128)
    assert torch.equal(fc1t[:, :120], bf(sd["fc1.weight"].t()))


def test_conv_fwd_matches_torch(env):
    nat, dev, ds, ref, tr = env
    n = 256
    s = _stream()
    nat.lenet_conv_fwd(s, tr.test_set.x.data_ptr(), 0, n, tr.pk.data_ptr(), tr.params.data_ptr(), 0,
                       tr.round_ctr.data_ptr(), 0, tr.act2.data_ptr(), 0, 0, 0, 0, 0)
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


@pytest.mark.parametrize("start,nb,augment", [(0, 128, True), (256, 128, False), (896, 80, True), (128, 33, True)])
def test_step_gradients_match_autograd(env, start, nb, augment):
    nat, dev, ds, ref, tr = env
    tr.load_state_dict(ref.state_dict())
    tr.round_ctr.zero_()
    g, dact2, stats = _run_grad(nat, tr, start, nb, augment)
    gr, out, loss, y = _ref_grad(ref, ds, start, nb, augment)
    off = 0
    for name, shape in LENET_SPEC:
        k = int(np.prod(shape))
        e = rel(g[off:off + k], gr[off:off + k])
        assert e < 5e-2, f"{name}: rel err {e:.3e}"
        off += k
    assert rel(g, gr) < 3e-2
    st = stats.cpu()
    assert int(st[2]) == nb
    loss_k = float(st[0:1].view(torch.float32)) / nb
    assert abs(loss_k - loss.item()) < 1e-2 * max(1.0, loss.item())
    assert abs(int(st[1]) - (out.argmax(1) == y).sum().item()) <= max(2, nb // 25)


def test_sgd_kernel_exact(env):
    nat, dev, ds, ref, tr = env
    L = tr.L
    torch.manual_seed(5)
    p0 = torch.randn(L["P_TOTAL"], device=dev)
    m0 = torch.randn(L["P_TOTAL"], device=dev) * 0.1
    tr.params.copy_(p0)
    tr.mom.copy_(m0)
    nb = 100
    nfc = 4
    tr.conv_slab.normal_()
    tr.fc_slab.normal_()
    nat.lenet_sgd(_stream(), tr.params.data_ptr(), tr.mom.data_ptr(), tr.pk.data_ptr(), tr.conv_slab.data_ptr(), nb,
                  tr.fc_slab.data_ptr(), nfc, 0.1, 0.9, 5e-4, 0)
    torch.cuda.synchronize()
    g = torch.cat([tr.conv_slab[:nb].double().sum(0), tr.fc_slab[:nfc].double().sum(0)])
    d = g + 5e-4 * p0.double()
    b = 0.9 * m0.double() + d
    p = p0.double() - 0.1 * b
    assert torch.allclose(tr.mom.double(), b, rtol=1e-5, atol=1e-5)
    assert torch.allclose(tr.params.double(), p, rtol=1e-5, atol=1e-5)
    # packed images follow the master weights
    pk = tr.pk.float()
    assert torch.equal(pk[:6 * 96].view(6, 96)[:, :75], tr.params[:450].view(6, 75).bfloat16().float())
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
    assert rel(pg - p0, pr - p0) < 6e-2


def test_training_converges(env):
    nat, dev, ds, ref, tr = env
    tr.load_state_dict(ref.state_dict())
    tr.mom.zero_()
    tr.cfg.use_graph = True
    tr.set_schedule(*strided_schedule(1024, 128, 0, 1))
    tr.set_schedule([], [])
    tr.set_schedule(*strided_schedule(1024, 128, 0, 1))
    for _ in range(6):
        tr.train_epoch()
    tr.evaluate()
    st = tr.eval_stats()
    assert st.acc > 50.0, st
