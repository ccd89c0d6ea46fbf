"""Fused SGD + weight images (conv.SgdPack, sgd_pack_kernel) against the unfused tail it replaces.

The fused launch must be bit-identical to ``sgd_flat`` followed by ``pack_weights`` and
``dgrad_pack_weights``: the same fp32 update (fedmi::sgd_elem, shared by both kernels) rounded to bf16
the same way.  Checked on a synthetic flat master (3x3 / 1x1 / 5x5 filters, stride 1 and 2, a padded
3-channel input, a 32-filter conv without a DGRAD image, non-conv segments in between) and on whole
engines: one step of ResNet-18 / MobileNet / GoogLeNet / VGG11 with the fused tail vs the unfused tail.
"""
import pytest
import torch

from fedmi import native
from fedmi.ops import conv

pytestmark = pytest.mark.gpu

# (O, Cw, R, S, stride, pad, dgrad image)
CONVS = [(64, 3, 3, 3, 1, 1, False), (64, 64, 3, 3, 1, 1, True), (128, 64, 3, 3, 2, 1, True),
         (128, 64, 1, 1, 2, 0, True), (32, 24, 5, 5, 1, 2, False), (64, 40, 5, 5, 2, 2, True),
         (512, 256, 3, 3, 1, 1, True), (64, 200, 1, 1, 1, 0, True), (24, 16, 1, 1, 1, 0, False)]


def _flat_master(dev):
    g = torch.Generator().manual_seed(0)
    sizes, gaps = [], []
    for i, (O, Cw, R, S, *_rest) in enumerate(CONVS):
        gaps.append(37 + 5 * i)                 # BN affine / bias-like segments between the convs
        sizes.append(O * Cw * R * S)
    n = sum(sizes) + sum(gaps) + 11
    p = (torch.randn(n, generator=g) * 0.1).to(dev)
    gr = (torch.randn(n, generator=g) * 0.01).to(dev)
    m = (torch.randn(n, generator=g) * 0.01).to(dev)
    views, off = [], 0
    for (O, Cw, R, S, *_rest), sz, gap in zip(CONVS, sizes, gaps):
        off += gap
        views.append((off, (O, Cw, R, S)))
        off += sz
    return p, gr, m, views


def test_sgd_pack_matches_sgd_flat_and_packs(gpu_device):
    p, g, m, views = _flat_master(gpu_device)
    items_a, items_b = [], []
    imgs = []
    for (off, shp), (O, Cw, R, S, st, pad, has_wd) in zip(views, CONVS):
        C = conv.pad8(Cw)
        wr = [torch.zeros(O, R, S, C, dtype=torch.bfloat16, device=gpu_device) for _ in range(2)]
        wd = ([torch.zeros(conv.dgrad_image_numel(shp, C), dtype=torch.bfloat16, device=gpu_device)
               for _ in range(2)] if has_wd else [None, None])
        imgs.append((wr, wd))
        items_a.append((off, shp, wr[0], wd[0], st, pad, C))
        items_b.append((off, shp, wr[1], wd[1], st, pad, C))
    lr, mom, wdecay = 0.05, 0.9, 5e-4

    # unfused: sgd_flat over the whole master, then the two pack launches
    pa, ma = p.clone(), m.clone()
    native.require().sgd_flat(native.stream_handle(gpu_device), pa.data_ptr(), g.data_ptr(), ma.data_ptr(),
                              pa.numel(), lr, mom, wdecay, 0.0, False, False)
    conv.pack_weights([(pa[off:off + torch.Size(shp).numel()].view(shp), wr) for off, shp, wr, _, _, _, _ in items_a])
    conv.dgrad_pack_weights([(pa[off:off + torch.Size(shp).numel()].view(shp), wd, st, pad, C)
                             for off, shp, _, wd, st, pad, C in items_a if wd is not None])

    # fused
    pb, mb = p.clone(), m.clone()
    sp = conv.SgdPack(pb, g, mb, [(pb[off:off + torch.Size(shp).numel()].view(shp), wr, wd, st, pad, C)
                                  for off, shp, wr, wd, st, pad, C in items_b])
    assert sp.n_convs == len(CONVS) and sp.n_segs == len(CONVS) + 1
    sp.step(lr, mom, wdecay)
    torch.cuda.synchronize()

    assert torch.equal(pa, pb)
    assert torch.equal(ma, mb)
    for k, (wr, wd) in enumerate(imgs):
        assert torch.equal(wr[0], wr[1]), f"forward image of conv {k}"
        if wd[0] is not None:
            assert torch.equal(wd[0], wd[1]), f"DGRAD image of conv {k}"


def test_sgd_pack_rejects_foreign_weight(gpu_device):
    p = torch.zeros(1000, device=gpu_device)
    other = torch.zeros(64, 8, 1, 1, device=gpu_device)
    wr = torch.zeros(64, 1, 1, 8, dtype=torch.bfloat16, device=gpu_device)
    with pytest.raises(ValueError):
        conv.SgdPack(p, p.clone(), p.clone(), [(other, wr, None, 1, 0, 8)])


@pytest.mark.parametrize("name", ["ResNet18", "MobileNet", "GoogLeNet", "VGG11"])
def test_engine_step_fused_tail_is_bit_identical(gpu_device, name):
    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.cnn_native import CNNNativeTrainer
    from fedmi.engine.data import make_dataset

    nb = 32
    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=64, n_test=32, seed=0)
    cfg = TrainerConfig(batch_size=nb, augment=False, use_graph=False, lr=0.05)
    engines = []
    for fused in (True, False):
        torch.manual_seed(5)
        tr = CNNNativeTrainer(name, data, gpu_device, cfg)
        assert tr._sgdpack is not None
        if not fused:
            tr._sgdpack = None
        engines.append(tr)
    a, b = engines
    b.load_state_dict(a.state_dict())
    for tr in engines:
        tr.set_schedule([0, nb], [nb, nb])
        tr.train_epoch()
    torch.cuda.synchronize()
    assert torch.equal(a.fs.flat, b.fs.flat)
    assert torch.equal(a.fs.mom, b.fs.mom)
    for ua, ub in zip(a.units, b.units):
        if ua.wr is not None:
            assert torch.equal(ua.wr, ub.wr)
        if ua.wd is not None and id(ua) not in a._no_dgrad:
            assert torch.equal(ua.wd, ub.wd)
