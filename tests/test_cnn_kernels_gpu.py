"""Implicit-GEMM conv (fwd / dgrad / wgrad), BatchNorm fwd/bwd and the
classifier head vs PyTorch fp32 references on the same bf16-rounded inputs."""
import pytest
import torch
import torch.nn.functional as F

from fedmi.ops import cnn, conv

pytestmark = pytest.mark.gpu

# (N, H, W, Cw, O, R, stride, pad): ResNet-18 CIFAR shapes at reduced batch + edge cases
SHAPES = [
    (4, 32, 32, 3, 64, 3, 1, 1),       # stem (input padded 3 -> 8 channels)
    (4, 32, 32, 64, 64, 3, 1, 1),      # layer1
    (4, 32, 32, 64, 128, 3, 2, 1),     # layer2 downsample
    (4, 32, 32, 64, 128, 1, 2, 0),     # projection shortcut
    (8, 8, 8, 256, 512, 3, 2, 1),      # layer4 downsample
    (16, 4, 4, 512, 512, 3, 1, 1),     # layer4
    (3, 7, 5, 24, 40, 3, 1, 1),        # odd spatial, partial tiles
    (2, 9, 9, 16, 8, 5, 2, 2),         # 5x5 stride 2
    # GoogLeNet inception branches: C % 64 != 0 runs the forward on conv_tap<GEN> (several taps per K step)
    (4, 32, 32, 96, 128, 3, 1, 1),     # a3 3x3 branch
    (4, 16, 16, 48, 48, 3, 1, 1),      # a4 double-3x3 branch
    (4, 16, 16, 480, 192, 1, 1, 0),    # a4 1x1 (C % 64 == 32)
    (16, 4, 4, 160, 320, 3, 1, 1),     # small M, long K (split-K of the GEN path)
    # O % 64 != 0 at stride 1: the DGRAD runs on conv_tap<GEN> over dY (O input channels)
    (4, 32, 32, 192, 16, 1, 1, 0),     # a3 1x1 -> 16 (K = 16: one masked K step)
    (4, 32, 32, 16, 32, 3, 1, 1),      # a3 16 -> 32 3x3
    (4, 8, 8, 832, 48, 1, 1, 0),       # b5 1x1 -> 48
]


def _rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-6))


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _make(shape, dev, seed=0):
    N, H, W, Cw, O, R, st, pad = shape
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, Cw, H, W, generator=g).to(dev).bfloat16().float()
    w = (torch.randn(O, Cw, R, R, generator=g) / (Cw * R * R) ** 0.5).to(dev)
    wb = w.bfloat16().float()
    C = conv.pad8(Cw)
    xn = torch.zeros(N, H, W, C, dtype=torch.bfloat16, device=dev)
    xn[..., :Cw] = _nhwc(x).bfloat16()
    return x, w, wb, xn


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_conv_fwd_and_stats(gpu_device, shape):
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device)
    wr = conv.pack_weight(w)
    rep = conv.stats_buffer(O, gpu_device)
    y = conv.conv2d_fwd(xn, wr, st, pad, Cw=Cw, stats=rep)
    stats = conv.stats_total(rep)
    ref = F.conv2d(x, wb, stride=st, padding=pad)
    torch.cuda.synchronize()
    assert _rel(y.float(), _nhwc(ref)) < 1e-2
    yb = y.float()
    assert torch.allclose(stats[0], yb.sum((0, 1, 2)), rtol=1e-3, atol=1e-2)
    assert torch.allclose(stats[1], (yb * yb).sum((0, 1, 2)), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_conv_dgrad_wgrad(gpu_device, shape):
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device, seed=1)
    xr = x.clone().requires_grad_(True)
    wr_ = wb.clone().requires_grad_(True)
    out = F.conv2d(xr, wr_, stride=st, padding=pad)
    gy = torch.randn_like(out).bfloat16().float()
    out.backward(gy)
    dyn = _nhwc(gy).bfloat16()
    wpk = conv.pack_weight(w)
    dx = conv.conv2d_dgrad(dyn, wpk, xn.shape, st, pad, Cw=Cw)
    dw = conv.conv2d_wgrad(xn, dyn, R, R, st, pad, Cw=Cw)
    torch.cuda.synchronize()
    assert _rel(dx[..., :Cw].float(), _nhwc(xr.grad)) < 1e-2
    if Cw < dx.shape[-1]:   # padded input channels see zero weights
        assert float(dx[..., Cw:].float().abs().max()) == 0.0
    assert _rel(dw, wr_.grad) < 1e-2
    if conv.dgrad_eligible(O, st):   # tap-major DGRAD on the flipped weight image (stride 1: any O % 8 via GEN)
        wd = torch.full((conv.dgrad_image_numel(w.shape, xn.shape[-1]),), float("nan"), dtype=torch.bfloat16,
                        device=gpu_device)
        conv.dgrad_pack_weights([(w, wd, st, pad, xn.shape[-1])])
        dx2 = torch.full_like(dx, float("nan"))
        conv.conv2d_dgrad(dyn, wpk, xn.shape, st, pad, Cw=Cw, out=dx2, wd=wd)
        torch.cuda.synchronize()
        assert _rel(dx2[..., :Cw].float(), _nhwc(xr.grad)) < 1e-2
        assert _rel(dx2.float(), dx.float()) < 1e-2


def test_dgrad_tap_edge_shapes(gpu_device):
    # partial M tiles, 1x1 stride-2 (empty parity phases), 5x5 stride 2, odd spatial
    for shape in [(3, 7, 5, 24, 64, 3, 1, 1), (4, 9, 9, 64, 128, 1, 2, 0), (2, 9, 11, 16, 64, 5, 2, 2),
                  (5, 6, 6, 128, 64, 3, 2, 1)]:
        N, H, W, Cw, O, R, st, pad = shape
        x, w, wb, xn = _make(shape, gpu_device, seed=9)
        xr = x.clone().requires_grad_(True)
        out = F.conv2d(xr, wb, stride=st, padding=pad)
        gy = torch.randn_like(out).bfloat16().float()
        out.backward(gy)
        dyn = _nhwc(gy).bfloat16()
        C = xn.shape[-1]
        wd = torch.empty(conv.dgrad_image_numel(w.shape, C), dtype=torch.bfloat16, device=gpu_device)
        conv.dgrad_pack_weights([(w, wd, st, pad, C)])
        dx = torch.full_like(xn, float("nan"))
        conv.conv2d_dgrad(dyn, conv.pack_weight(w), xn.shape, st, pad, Cw=Cw, out=dx, wd=wd)
        torch.cuda.synchronize()
        assert not torch.isnan(dx.float()).any(), shape
        assert _rel(dx[..., :Cw].float(), _nhwc(xr.grad)) < 1e-2, shape
        if Cw < C:
            assert float(dx[..., Cw:].float().abs().max()) == 0.0


def test_conv_wgrad_split_invariance(gpu_device):
    shape = (8, 16, 16, 64, 64, 3, 1, 1)
    _, _, _, xn = _make(shape, gpu_device, seed=2)
    dy = torch.randn(8, 16, 16, 64, device=gpu_device).bfloat16()
    a = conv.conv2d_wgrad(xn, dy, 3, 3, 1, 1, splits=1)
    b = conv.conv2d_wgrad(xn, dy, 3, 3, 1, 1, splits=7)
    torch.cuda.synchronize()
    assert _rel(a, b) < 1e-4


@pytest.mark.parametrize("shape", [(128, 4, 4, 512, 512), (128, 2, 2, 1024, 1024), (16, 4, 4, 256, 512),
                                   (64, 8, 8, 128, 256)])
def test_conv_wgrad_1x1_library_route(gpu_device, shape, monkeypatch):
    """1x1 / stride-1 WGRAD over <= 2048 pixels goes to the library GEMM (conv.WGRAD_GEMM_PIXELS); both routes
    match fp32 and each other, and the library route is bit-stable run to run."""
    N, H, W, C, O = shape
    torch.manual_seed(11)
    xn = torch.randn(N, H, W, C, device=gpu_device).bfloat16()
    dy = torch.randn(N, H, W, O, device=gpu_device).bfloat16()
    ref = (dy.float().view(-1, O).t() @ xn.float().view(-1, C)).view(O, C, 1, 1)
    lib = conv.conv2d_wgrad(xn, dy, 1, 1, 1, 0)
    lib2 = conv.conv2d_wgrad(xn, dy, 1, 1, 1, 0)
    monkeypatch.setattr(conv, "WGRAD_GEMM_PIXELS", 0)
    nat = conv.conv2d_wgrad(xn, dy, 1, 1, 1, 0)
    torch.cuda.synchronize()
    assert _rel(lib, ref) < 1e-5 and _rel(nat, ref) < 1e-5
    assert torch.equal(lib, lib2)


@pytest.mark.parametrize("shape", [(8, 16, 16, 64, 128), (4, 32, 32, 192, 64), (16, 8, 8, 256, 256), (2, 8, 8, 128, 64),
                                   (128, 8, 8, 832, 256)])
def test_conv_wgrad_1x1_halo_kernel(gpu_device, shape, monkeypatch):
    """1x1 / stride-1 WGRAD with C, O % 64 (M (C + O) <= 12.6 M) runs on conv_wgrad_halo<1, 1> (the block's own
    pixel rows as the one-tap patch); against fp32 and the generic kernel (explicit splits, and lib_gemm=False --
    the aten backend's route -- both take it)."""
    N, H, W, C, O = shape
    torch.manual_seed(13)
    xn = torch.randn(N, H, W, C, device=gpu_device).bfloat16()
    dy = torch.randn(N, H, W, O, device=gpu_device).bfloat16()
    ref = (dy.float().view(-1, O).t() @ xn.float().view(-1, C)).view(O, C, 1, 1)
    monkeypatch.setattr(conv, "WGRAD_GEMM_PIXELS", 0)                         # no library route at small M
    dw = conv.conv2d_wgrad(xn, dy, 1, 1, 1, 0)
    dw1 = conv.conv2d_wgrad(xn, dy, 1, 1, 1, 0, splits=1)                     # explicit splits: generic kernel
    dw2 = conv.conv2d_wgrad(xn, dy, 1, 1, 1, 0, lib_gemm=False)               # generic, automatic splits
    torch.cuda.synchronize()
    assert _rel(dw2, ref) < 1e-4
    torch.cuda.synchronize()
    assert _rel(dw, ref) < 1e-4 and _rel(dw1, ref) < 1e-4
    assert _rel(dw, dw1) < 1e-4


def _bn_ref(z, gamma, beta, eps=1e-5):
    mean = z.mean(0)
    var = z.var(0, unbiased=False)
    return (z - mean) / torch.sqrt(var + eps) * gamma + beta, mean, var


def test_bn_forward_backward_with_projection_residual(gpu_device):
    torch.manual_seed(3)
    dev = gpu_device
    M, C = 4 * 16 * 16, 128
    za = (torch.randn(M, C, device=dev) * 2 + 0.5).bfloat16()
    zb = (torch.randn(M, C, device=dev) - 0.3).bfloat16()
    ga, ba = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    gb, bb = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    # replicated statistics buffers: the totals spread unevenly over the STAT_REP replicas
    wrep = torch.arange(1, conv.STAT_REP + 1, device=dev, dtype=torch.float64)
    wrep = (wrep / wrep.sum()).view(-1, 1, 1)
    sa = (torch.stack([za.double().sum(0), (za.double() ** 2).sum(0)]) * wrep).contiguous()
    sb = (torch.stack([zb.double().sum(0), (zb.double() ** 2).sum(0)]) * wrep).contiguous()
    rma, rva, rmb, rvb = (torch.zeros(C, device=dev), torch.ones(C, device=dev),
                          torch.zeros(C, device=dev), torch.ones(C, device=dev))
    nbt = torch.zeros(1, dtype=torch.int64, device=dev)
    sma, sia, smb, sib = (torch.empty(C, device=dev) for _ in range(4))
    A = cnn.bn_desc(sa, ga, ba, rma, rva, nbt, sma, sia)
    B = cnn.bn_desc(sb, gb, bb, rmb, rvb, None, smb, sib)
    y = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    cnn.bn_apply(za, A, y, train=True, relu=True, z2=zb, b=B)
    # reference
    zar, zbr = za.float().requires_grad_(True), zb.float().requires_grad_(True)
    gar, gbr = ga.clone().requires_grad_(True), gb.clone().requires_grad_(True)
    bar, bbr = ba.clone().requires_grad_(True), bb.clone().requires_grad_(True)
    ya, mean_a, var_a = _bn_ref(zar, gar, bar)
    yb, _, _ = _bn_ref(zbr, gbr, bbr)
    yref = F.relu(ya + yb)
    torch.cuda.synchronize()
    assert _rel(y.float(), yref) < 1e-2
    assert torch.allclose(rma, 0.1 * mean_a.detach(), atol=1e-4)
    assert torch.allclose(rva, 0.9 + 0.1 * var_a.detach() * M / (M - 1), rtol=1e-3)
    assert int(nbt.item()) == 1
    # backward with a residual fan-in (dya + dyb)
    dya = torch.randn(M, C, device=dev).bfloat16()
    dyb = torch.randn(M, C, device=dev).bfloat16()
    yref.backward(dya.float() + dyb.float())
    dza, dzb, gout = (torch.empty(M, C, dtype=torch.bfloat16, device=dev) for _ in range(3))
    dga, dba, dgb, dbb = (torch.empty(C, device=dev) for _ in range(4))
    red = torch.zeros(3, C, dtype=torch.float64, device=dev)
    cnn.bn_bwd(dya, za, A, dga, dba, dza, red, dyb=dyb, y=y, zb=zb, b=B, dgamma_b=dgb, dbeta_b=dbb, dzb=dzb,
               gout=gout)
    torch.cuda.synchronize()
    assert _rel(dza.float(), zar.grad) < 2e-2
    assert _rel(dzb.float(), zbr.grad) < 2e-2
    assert _rel(dga, gar.grad) < 1e-2 and _rel(dba, bar.grad) < 1e-2
    assert _rel(dgb, gbr.grad) < 1e-2 and _rel(dbb, bbr.grad) < 1e-2
    mask = (y.float() > 0).float()
    assert _rel(gout.float(), (dya.float() + dyb.float()) * mask) < 1e-2
    # two-level reduction (replicated atomics + finalize): same result, red needs no init, ws left zero
    ws = torch.zeros(cnn.bn_bwd_ws_floats(M, C), dtype=torch.float64, device=dev)
    red2 = torch.full((3, C), float("nan"), dtype=torch.float64, device=dev)
    dza2, dzb2 = torch.empty_like(dza), torch.empty_like(dzb)
    dga2, dba2, dgb2, dbb2 = (torch.empty(C, device=dev) for _ in range(4))
    for _ in range(2):   # the scratch is reusable without re-zeroing
        cnn.bn_bwd(dya, za, A, dga2, dba2, dza2, red2, dyb=dyb, y=y, zb=zb, b=B, dgamma_b=dgb2, dbeta_b=dbb2,
                   dzb=dzb2, ws=ws)
        first = dga2.clone() if _ == 0 else first
    torch.cuda.synchronize()
    assert _rel(first, dga2) < 1e-5 and float(ws.abs().max()) == 0.0
    assert _rel(dza2.float(), dza.float()) < 1e-2 and _rel(dzb2.float(), dzb.float()) < 1e-2
    assert _rel(dga2, dga) < 1e-4 and _rel(dba2, dba) < 1e-4 and _rel(dgb2, dgb) < 1e-4
    # chained mode (the engine's default): per-BN replicas read by the apply kernel, no finalize launch,
    # no 'red' use at all; the replicas must be zero on entry (the head launch clears them per step)
    rep = torch.zeros(cnn.bn_bwd_chain_floats(C), dtype=torch.float64, device=dev)
    red3 = torch.full((3, C), float("nan"), dtype=torch.float64, device=dev)
    dza3, dzb3 = torch.empty_like(dza), torch.empty_like(dzb)
    dga3, dba3, dgb3, dbb3 = (torch.empty(C, device=dev) for _ in range(4))
    cnn.bn_bwd(dya, za, A, dga3, dba3, dza3, red3, dyb=dyb, y=y, zb=zb, b=B, dgamma_b=dgb3, dbeta_b=dbb3,
               dzb=dzb3, ws=rep, chained=True)
    torch.cuda.synchronize()
    assert _rel(dza3.float(), dza.float()) < 1e-2 and _rel(dzb3.float(), dzb.float()) < 1e-2
    assert _rel(dga3, dga) < 1e-4 and _rel(dba3, dba) < 1e-4 and _rel(dgb3, dgb) < 1e-4 and _rel(dbb3, dbb) < 1e-4
    # the head launch clears a replica arena
    rep2 = torch.ones(64, device=dev)
    Nh, Ch = 4, 64
    cnn.head(torch.randn(Nh, 2, 2, Ch, device=dev).bfloat16(), torch.zeros(Nh, dtype=torch.int32, device=dev), 0,
             torch.randn(10, Ch, device=dev), torch.zeros(10, device=dev), torch.zeros(4, device=dev), False,
             zero=rep2)
    torch.cuda.synchronize()
    assert float(rep2.abs().max()) == 0.0


def test_bn_eval_uses_running_stats(gpu_device):
    dev = gpu_device
    M, C = 64, 64
    z = torch.randn(M, C, device=dev).bfloat16()
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    rm, rv = torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5
    y = torch.empty_like(z)
    res = torch.randn(M, C, device=dev).bfloat16()
    cnn.bn_apply(z, cnn.bn_desc(None, g, b, rm, rv), y, train=False, relu=False, res=res)
    ref = (z.float() - rm) / torch.sqrt(rv + 1e-5) * g + b + res.float()
    torch.cuda.synchronize()
    assert _rel(y.float(), ref) < 1e-2


def test_head_ce_and_grads(gpu_device):
    torch.manual_seed(4)
    dev = gpu_device
    N, HW, C, J = 16, 16, 512, 10
    y = torch.randn(N, 4, 4, C, device=dev).bfloat16()
    labels = torch.randint(0, J, (N,), device=dev, dtype=torch.int32)
    W = torch.randn(J, C, device=dev) * 0.05
    b = torch.randn(J, device=dev) * 0.1
    stats = torch.zeros(4, device=dev)
    pooled = torch.empty(N, C, device=dev)
    dlog = torch.empty(N, J, device=dev)
    dy = torch.empty_like(y)
    dW = torch.empty(J, C, device=dev)
    db = torch.empty(J, device=dev)
    cnn.head(y, labels, 0, W, b, stats, True, pooled, dlog, dy, dW, db)
    yr = y.float().requires_grad_(True)
    Wr, br = W.clone().requires_grad_(True), b.clone().requires_grad_(True)
    logits = F.linear(yr.mean((1, 2)), Wr, br)
    loss = F.cross_entropy(logits, labels.long())
    loss.backward()
    torch.cuda.synchronize()
    s = stats.view(torch.int32)
    assert abs(float(stats[0]) / N - float(loss)) < 1e-3
    assert int(s[1]) == int((logits.argmax(1) == labels.long()).sum()) and int(s[2]) == N
    assert _rel(dW, Wr.grad) < 1e-4 and _rel(db, br.grad) < 1e-4
    assert _rel(dy.float(), yr.grad) < 1e-2


def test_prep_input_matches_host_twin(gpu_device):
    from fedmi.engine.data import augment_normalize
    import numpy as np

    dev = gpu_device
    imgs = torch.randint(0, 256, (10, 3, 32, 32), dtype=torch.uint8, device=dev)
    rc = torch.tensor([3, 0, 0, 0], dtype=torch.int32, device=dev)
    out = cnn.prep_input(imgs, 2, 6, True, 1234, rc)
    ref = augment_normalize(imgs[2:8], np.arange(2, 8), 1234, 3)
    torch.cuda.synchronize()
    assert torch.allclose(out[..., :3].float(), _nhwc(ref), atol=2e-2)
    assert float(out[..., 3:].float().abs().max()) == 0.0


DW_SHAPES = [(4, 32, 32, 32, 3, 1), (4, 32, 32, 64, 3, 2), (8, 4, 4, 1024, 3, 1), (2, 16, 16, 96, 5, 2),
             (2, 8, 8, 16, 7, 1),
             # batch-128 MobileNet / MobileNetV2 layers where the wgrad splits channels into chunks
             # (C/8 = 128, 64, 120 -> chunks of 32, 32, 30; 48 -> 24)
             (128, 2, 2, 1024, 3, 1), (128, 4, 4, 512, 3, 1), (128, 4, 4, 960, 3, 1), (128, 8, 8, 384, 3, 1),
             # odd output widths: the row-pair 3x3 forward's unpaired last column
             (3, 7, 7, 64, 3, 1), (2, 9, 9, 32, 3, 2)]


@pytest.mark.parametrize("shape", DW_SHAPES, ids=[str(s) for s in DW_SHAPES])
def test_depthwise_fwd_dgrad_wgrad(gpu_device, shape):
    N, H, W, C, R, st = shape
    pad = R // 2
    dev = gpu_device
    torch.manual_seed(5)
    x = torch.randn(N, C, H, W, device=dev).bfloat16().float().requires_grad_(True)
    w = (torch.randn(C, 1, R, R, device=dev) * 0.2)
    wb = w.bfloat16().float().requires_grad_(True)
    ref = F.conv2d(x, w, stride=st, padding=pad, groups=C)
    gy = torch.randn_like(ref).bfloat16().float()
    ref.backward(gy)
    wref = F.conv2d(x.detach(), wb, stride=st, padding=pad, groups=C)
    wref.backward(gy)
    xn = _nhwc(x.detach()).bfloat16()
    rep = conv.stats_buffer(C, dev)
    y = conv.dwconv_fwd(xn, w, st, pad, stats=rep)
    stats = conv.stats_total(rep)
    dx = conv.dwconv_dgrad(_nhwc(gy).bfloat16(), w, xn.shape, st, pad)
    dw = conv.dwconv_wgrad(xn, _nhwc(gy).bfloat16(), R, st, pad)
    torch.cuda.synchronize()
    assert _rel(y.float(), _nhwc(ref.detach())) < 1e-2
    yb = y.float()
    assert torch.allclose(stats[0], yb.sum((0, 1, 2)), rtol=1e-3, atol=1e-2)
    assert _rel(dx.float(), _nhwc(x.grad)) < 1e-2
    assert _rel(dw, wb.grad) < 1e-2


def test_bn_backward_relu_mask_from_z(gpu_device):
    """A ReLU'd BN inside a block: bn_apply records the scale / shift it applied (co_out) and the BN backward
    derives the ReLU mask from z (z * scale + shift > 0) instead of re-reading the materialised y."""
    dev = gpu_device
    torch.manual_seed(9)
    N, H, W, C = 8, 8, 8, 256
    z = torch.randn(N, H, W, C, device=dev).bfloat16()
    # BN backward: mask from z == mask from the materialised y
    M = N * H * W
    zr = z.reshape(M, C)
    stats = conv.stats_buffer(C, dev)
    stats.zero_()
    stats[0, 0].copy_(zr.float().sum(0))
    stats[0, 1].copy_((zr.float() ** 2).sum(0))
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
    A = cnn.bn_desc(stats, g, b, None, None, None, sm, si)
    co2 = torch.empty(2, C, device=dev)
    yb = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    cnn.bn_apply(zr, A, yb, train=True, relu=True, co_out=co2)
    torch.cuda.synchronize()
    assert _rel(torch.relu(zr.float() * co2[0] + co2[1]), yb.float()) < 1e-2
    dya = torch.randn(M, C, device=dev).bfloat16()
    outs = []
    for use_mask in (False, True):
        dz = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
        dg, db_ = torch.empty(C, device=dev), torch.empty(C, device=dev)
        red = torch.zeros(3, C, dtype=torch.float64, device=dev)
        if use_mask:
            cnn.bn_bwd(dya, zr, A, dg, db_, dz, red, mask_bn=co2)
        else:
            cnn.bn_bwd(dya, zr, A, dg, db_, dz, red, y=yb)
        outs.append((dz.float(), dg.clone(), db_.clone()))
    torch.cuda.synchronize()
    (dz0, dg0, db0), (dz1, dg1, db1) = outs
    # y is bf16-rounded: a value at the ReLU edge may flip; everything else is identical math
    assert _rel(dz1, dz0) < 1e-2 and _rel(dg1, dg0) < 1e-2 and _rel(db1, db0) < 1e-2


# full-batch ResNet-18 layer3/4 shapes: few output tiles + long K -> split-K through a workspace
SPLIT_SHAPES = [
    (128, 8, 8, 256, 256, 3, 1, 1),     # layer3
    (128, 4, 4, 512, 512, 3, 1, 1),     # layer4
    (128, 8, 8, 256, 512, 3, 2, 1),     # layer4 downsample (stride-2 dgrad phases)
]


@pytest.mark.parametrize("shape", SPLIT_SHAPES, ids=[str(s) for s in SPLIT_SHAPES])
def test_conv_splitk_fwd_dgrad(gpu_device, shape):
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device, seed=4)
    wr = conv.pack_weight(w)
    need = conv.fd_ws_floats(xn.shape, O, R, R, st, pad, Cw)
    assert need > 0, "shape expected to take the split-K path"
    ws = torch.full((need,), float("nan"), device=gpu_device)   # every partial must be written
    shift = torch.randn(O, device=gpu_device) * 0.1
    r_split, r_one = conv.stats_buffer(O, gpu_device), conv.stats_buffer(O, gpu_device)
    y = conv.conv2d_fwd(xn, wr, st, pad, Cw=Cw, stats=r_split, shift=shift, ws=ws)
    y1 = conv.conv2d_fwd(xn, wr, st, pad, Cw=Cw, stats=r_one, shift=shift)
    s_split = conv.stats_total(r_split)
    ref = F.conv2d(x, wb, stride=st, padding=pad)
    torch.cuda.synchronize()
    assert _rel(y.float(), _nhwc(ref)) < 1e-2
    assert _rel(y.float(), y1.float()) < 1e-2
    d = y.float() - shift
    assert torch.allclose(s_split[0], d.sum((0, 1, 2)), rtol=1e-3, atol=1e-1)
    assert torch.allclose(s_split[1], (d * d).sum((0, 1, 2)), rtol=1e-3, atol=1e-1)
    # data gradient
    xr = x.clone().requires_grad_(True)
    out = F.conv2d(xr, wb, stride=st, padding=pad)
    gy = torch.randn_like(out).bfloat16().float()
    out.backward(gy)
    dyn = _nhwc(gy).bfloat16()
    ws.fill_(float("nan"))
    dx = conv.conv2d_dgrad(dyn, wr, xn.shape, st, pad, Cw=Cw, ws=ws)
    torch.cuda.synchronize()
    assert _rel(dx.float(), _nhwc(xr.grad)) < 1e-2
    wd = torch.empty(conv.dgrad_image_numel(w.shape, xn.shape[-1]), dtype=torch.bfloat16, device=gpu_device)
    conv.dgrad_pack_weights([(w, wd, st, pad, xn.shape[-1])])
    ws.fill_(float("nan"))
    dx2 = conv.conv2d_dgrad(dyn, wr, xn.shape, st, pad, Cw=Cw, ws=ws, wd=wd)
    torch.cuda.synchronize()
    assert _rel(dx2.float(), _nhwc(xr.grad)) < 1e-2


def test_conv_wgrad_many_splits_and_padded_channels(gpu_device):
    # stem-like: 3 real channels padded to 8, deep K (many splits): the parallel reduce + permute
    shape = (64, 32, 32, 3, 64, 3, 1, 1)
    x, w, wb, xn = _make(shape, gpu_device, seed=5)
    xr = x.clone()
    wr_ = wb.clone().requires_grad_(True)
    out = F.conv2d(xr, wr_, stride=1, padding=1)
    gy = torch.randn_like(out).bfloat16().float()
    out.backward(gy)
    dyn = _nhwc(gy).bfloat16()
    for sp in (0, 1, 37, 128):
        dw = conv.conv2d_wgrad(xn, dyn, 3, 3, 1, 1, Cw=3, splits=sp)
        torch.cuda.synchronize()
        assert _rel(dw, wr_.grad) < 1e-2, sp
    base = torch.randn(64, 3, 3, 3, device=gpu_device)
    acc = conv.conv2d_wgrad(xn, dyn, 3, 3, 1, 1, Cw=3, out=base.clone(), accumulate=True)
    torch.cuda.synchronize()
    assert _rel(acc - base, wr_.grad) < 1e-2


def test_pack_weights_multi(gpu_device):
    torch.manual_seed(6)
    ws = [torch.randn(o, c, r, r, device=gpu_device) for o, c, r in ((64, 3, 3), (128, 64, 1), (16, 24, 5))]
    single = [conv.pack_weight(w) for w in ws]
    multi = [torch.full_like(s, 7.0) for s in single]
    conv.pack_weights(list(zip(ws, multi)))
    torch.cuda.synchronize()
    for a, b in zip(single, multi):
        assert torch.equal(a, b)


def test_maxpool2_fwd_bwd(gpu_device):
    torch.manual_seed(11)
    x = torch.randn(6, 8, 10, 24, device=gpu_device).bfloat16()
    y = cnn.maxpool2(x)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.max_pool2d(xr, 2, 2)
    g = torch.randn_like(ref).bfloat16().float()
    ref.backward(g)
    dx = cnn.maxpool2_bwd(x, _nhwc(g).bfloat16().contiguous())
    torch.cuda.synchronize()
    assert torch.equal(y.float(), _nhwc(ref.detach()))
    assert torch.equal(dx.float(), _nhwc(xr.grad))


def test_bn_conv_bias_folding(gpu_device):
    """BN(z + b) with b kept out of z: same train output, running_mean includes b, eval uses it."""
    torch.manual_seed(12)
    dev = gpu_device
    M, C = 512, 64
    z = torch.randn(M, C, device=dev).bfloat16()
    b = torch.randn(C, device=dev)
    g, be = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    rep = conv.stats_buffer(C, dev)
    rep[0, 0] = z.float().sum(0)
    rep[0, 1] = (z.float() ** 2).sum(0)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
    y = torch.empty_like(z)
    cnn.bn_apply(z, cnn.bn_desc(rep, g, be, rm, rv, None, sm, si, cbias=b), y, train=True, relu=False)
    zb = z.float() + b
    mean, var = zb.mean(0), zb.var(0, unbiased=False)
    ref = (zb - mean) / torch.sqrt(var + 1e-5) * g + be
    torch.cuda.synchronize()
    assert _rel(y.float(), ref) < 1e-2
    assert torch.allclose(rm, 0.1 * mean, atol=1e-4)
    ye = torch.empty_like(z)
    cnn.bn_apply(z, cnn.bn_desc(None, g, be, rm, rv, cbias=b), ye, train=False, relu=False)
    refe = (zb - rm) / torch.sqrt(rv + 1e-5) * g + be
    torch.cuda.synchronize()
    assert _rel(ye.float(), refe) < 1e-2


@pytest.mark.parametrize("shape", [(16, 16, 16, 64, 64, 3, 1, 1), (128, 4, 4, 512, 512, 3, 1, 1)],
                         ids=["single", "splitk"])
def test_conv_fwd_fused_residual(gpu_device, shape):
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device, seed=13)
    wr = conv.pack_weight(w)
    ref = _nhwc(F.conv2d(x, wb, stride=st, padding=pad))
    res = torch.randn_like(ref).bfloat16()
    shp = (xn.shape, O, R, R, st, pad, Cw)
    ws = torch.empty(max(conv.fd_ws_floats(*shp), 1), device=gpu_device)
    rep = conv.stats_buffer(O, gpu_device)
    y = conv.conv2d_fwd(xn, wr, st, pad, Cw=Cw, stats=rep, ws=ws, res=res)
    torch.cuda.synchronize()
    want = ref + res.float()
    assert _rel(y.float(), want) < 1e-2
    tot = conv.stats_total(rep)
    yb = y.float()
    assert torch.allclose(tot[0], yb.sum((0, 1, 2)), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("stride,shape,ties", [(1, (4, 9, 7, 24), False), (2, (3, 16, 16, 64), False),
                                               (2, (2, 9, 11, 16), False), (1, (2, 32, 32, 16), True),
                                               (1, (3, 6, 5, 8), True), (2, (2, 15, 13, 8), True)])
def test_maxpool3_fwd_bwd_accumulate(gpu_device, stride, shape, ties):
    """MaxPool2d(3, stride, 1) (GoogLeNet) vs torch: forward, gather backward (overlapping windows sum), +=.
    ``ties``: values on a coarse grid, so windows hold equal maxima -- the first maximum in (r, s) order must win,
    as in max_pool2d_with_indices (the register-blocked kernels scan each window in that order)."""
    torch.manual_seed(15)
    x = torch.randn(*shape, device=gpu_device)
    if ties:
        x = torch.round(x * 2) / 2
    x = x.bfloat16()
    y, idx = cnn.maxpool3(x, stride)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.max_pool2d(xr, 3, stride, 1)
    g = torch.randn_like(ref).bfloat16().float()
    ref.backward(g)
    base = torch.randn_like(x)
    dx = cnn.maxpool3_bwd(_nhwc(g).bfloat16(), idx, x.shape, stride, out=base.clone(), accumulate=True)
    dx0 = cnn.maxpool3_bwd(_nhwc(g).bfloat16(), idx, x.shape, stride)
    torch.cuda.synchronize()
    assert torch.equal(y.float(), _nhwc(ref.detach()))
    assert _rel(dx0.float(), _nhwc(xr.grad)) < 1e-2
    assert _rel(dx.float() - base.float(), _nhwc(xr.grad)) < 2e-2


def test_bn_strided_channel_slices(gpu_device):
    """bn_apply writing, and bn_bwd reading, a channel slice of a wider NHWC buffer (concat outputs)."""
    torch.manual_seed(16)
    dev = gpu_device
    M, C, W, off = 768, 48, 160, 64
    z = torch.randn(M, C, device=dev).bfloat16()
    g, be = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    rep = conv.stats_buffer(C, dev)
    rep[0, 0], rep[0, 1] = z.float().sum(0), (z.float() ** 2).sum(0)
    sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
    A = cnn.bn_desc(rep, g, be, None, None, None, sm, si)
    wide = torch.full((M, W), 7.0, device=dev).bfloat16()
    ys = wide[:, off:off + C]
    cnn.bn_apply(z, A, ys, train=True, relu=True)
    yc = torch.empty_like(z)
    cnn.bn_apply(z, A, yc, train=True, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(ys.float(), yc.float())
    assert float((wide[:, :off].float() - 7).abs().max()) == 0 and float((wide[:, off + C:].float() - 7).abs().max()) == 0
    dwide = torch.randn(M, W, device=dev).bfloat16()
    red = torch.empty(3, C, dtype=torch.float64, device=dev)
    ws = torch.zeros(cnn.bn_bwd_ws_floats(M, C), dtype=torch.float64, device=dev)
    d1, d2 = torch.empty_like(z), torch.empty_like(z)
    dg1, db1, dg2, db2 = (torch.empty(C, device=dev) for _ in range(4))
    cnn.bn_bwd(dwide[:, off:off + C], z, A, dg1, db1, d1, red, y=ys, ws=ws)
    cnn.bn_bwd(dwide[:, off:off + C].contiguous(), z, A, dg2, db2, d2, red, y=yc, ws=ws)
    torch.cuda.synchronize()
    assert torch.equal(d1, d2) and torch.allclose(dg1, dg2, rtol=1e-5, atol=1e-4) and torch.allclose(db1, db2)


@pytest.mark.parametrize("shape", [(4, 16, 16, 64, 64, 3, 1, 1), (8, 8, 8, 128, 64, 1, 1, 0),
                                   (4, 16, 16, 64, 128, 3, 2, 1), (3, 7, 5, 24, 40, 3, 1, 1)])
def test_conv_dgrad_accumulate(gpu_device, shape):
    """dx += DGRAD (fan-in of a multi-branch block), tap-major and generic paths, with split-K."""
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device, seed=17)
    xr = x.clone().requires_grad_(True)
    out = F.conv2d(xr, wb, stride=st, padding=pad)
    gy = torch.randn_like(out).bfloat16().float()
    out.backward(gy)
    dyn = _nhwc(gy).bfloat16()
    wpk = conv.pack_weight(w)
    C = xn.shape[-1]
    shp = (xn.shape, O, R, R, st, pad, Cw)
    wsp = torch.empty(max(conv.fd_ws_floats(*shp), 1), device=gpu_device)
    wds = [None]
    if conv.dgrad_eligible(O, st):
        wd = torch.empty(conv.dgrad_image_numel(w.shape, C), dtype=torch.bfloat16, device=gpu_device)
        conv.dgrad_pack_weights([(w, wd, st, pad, C)])
        wds.append(wd)
    for wd in wds:
        base = (torch.randn_like(xn.float()) * 0.05).bfloat16()
        dx = conv.conv2d_dgrad(dyn, wpk, xn.shape, st, pad, Cw=Cw, out=base.clone(), ws=wsp, wd=wd, accumulate=True)
        torch.cuda.synchronize()
        assert _rel(dx[..., :Cw].float() - base[..., :Cw].float(), _nhwc(xr.grad)) < 2e-2, wd is not None


def test_bn_bwd_additive_residual_grad(gpu_device):
    torch.manual_seed(14)
    dev = gpu_device
    M, C = 1024, 64
    z = torch.randn(M, C, device=dev).bfloat16()
    g, be = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    rep = conv.stats_buffer(C, dev)
    rep[0, 0], rep[0, 1] = z.float().sum(0), (z.float() ** 2).sum(0)
    sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
    A = cnn.bn_desc(rep, g, be, None, None, None, sm, si)
    y = torch.empty_like(z)
    cnn.bn_apply(z, A, y, train=True, relu=True)
    dy = torch.randn(M, C, device=dev).bfloat16()
    extra = torch.randn(M, C, device=dev).bfloat16()
    d1, d2 = torch.empty_like(z), torch.empty_like(z)
    dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
    ws = torch.zeros(cnn.bn_bwd_ws_floats(M, C), dtype=torch.float64, device=dev)
    red = torch.empty(3, C, dtype=torch.float64, device=dev)
    cnn.bn_bwd(dy, z, A, dg, db, d1, red, y=y, ws=ws)
    cnn.bn_bwd(dy, z, A, dg, db, d2, red, y=y, ws=ws, dadd=extra)
    torch.cuda.synchronize()
    assert _rel(d2.float() - extra.float(), d1.float()) < 2e-2


# The exact batch-128 ResNet-18 (CIFAR) conv shapes of SURVEY.md §2.4(b), run the way the engine runs
# them: forward with the split-K workspace and fused BN statistics, tap-major DGRAD on the weight
# image (+ workspace), auto-split WGRAD.
R18_B128 = [
    (128, 32, 32, 3, 64, 3, 1, 1),      # stem (input padded 3 -> 8 channels)
    (128, 32, 32, 64, 64, 3, 1, 1),     # layer1 (x4)
    (128, 32, 32, 64, 128, 3, 2, 1),    # layer2.0.conv1
    (128, 16, 16, 128, 128, 3, 1, 1),   # layer2
    (128, 32, 32, 64, 128, 1, 2, 0),    # layer2.0 shortcut
    (128, 16, 16, 128, 256, 3, 2, 1),   # layer3.0.conv1
    (128, 8, 8, 256, 256, 3, 1, 1),     # layer3
    (128, 16, 16, 128, 256, 1, 2, 0),   # layer3.0 shortcut
    (128, 8, 8, 256, 512, 3, 2, 1),     # layer4.0.conv1
    (128, 4, 4, 512, 512, 3, 1, 1),     # layer4
    (128, 8, 8, 256, 512, 1, 2, 0),     # layer4.0 shortcut
]


@pytest.mark.parametrize("shape", R18_B128, ids=[str(s) for s in R18_B128])
def test_resnet18_batch128_conv_shapes(gpu_device, shape):
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device, seed=3)
    xr = x.clone().requires_grad_(True)
    wr_ = wb.clone().requires_grad_(True)
    ref = F.conv2d(xr, wr_, stride=st, padding=pad)
    gy = torch.randn_like(ref).bfloat16().float()
    ref.backward(gy)
    C = xn.shape[-1]
    shp = (xn.shape, O, R, R, st, pad, Cw)
    ws = conv.wgrad_workspace(gpu_device, max(conv.fd_ws_floats(*shp), conv.wgrad_ws_floats(*shp), 1))
    wpk = conv.pack_weight(w)
    rep = conv.stats_buffer(O, gpu_device)
    y = conv.conv2d_fwd(xn, wpk, st, pad, Cw=Cw, stats=rep, ws=ws)
    dyn = _nhwc(gy).bfloat16()
    wd = None
    if conv.dgrad_eligible(O, st):
        wd = torch.empty(conv.dgrad_image_numel(w.shape, C), dtype=torch.bfloat16, device=gpu_device)
        conv.dgrad_pack_weights([(w, wd, st, pad, C)])
    dx = conv.conv2d_dgrad(dyn, wpk, xn.shape, st, pad, Cw=Cw, ws=ws, wd=wd)
    dw = conv.conv2d_wgrad(xn, dyn, R, R, st, pad, Cw=Cw, ws=ws)
    torch.cuda.synchronize()
    assert _rel(y.float(), _nhwc(ref.detach())) < 1e-2
    stats = conv.stats_total(rep)
    yb = y.float()
    assert _rel(stats[0], yb.sum((0, 1, 2))) < 1e-3
    assert _rel(stats[1], (yb * yb).sum((0, 1, 2))) < 1e-3
    assert _rel(dx[..., :Cw].float(), _nhwc(xr.grad)) < 1e-2
    assert _rel(dw, wr_.grad) < 1e-2


@pytest.mark.parametrize("shape", [(4, 32, 32, 64, 64, 3, 1, 1), (8, 16, 16, 128, 64, 3, 1, 1),
                                   (16, 8, 8, 64, 192, 3, 1, 1), (128, 32, 32, 64, 64, 3, 1, 1),
                                   (128, 8, 8, 256, 256, 3, 1, 1)],
                         ids=["w32", "w16", "w8_o192", "l1_b128", "l3_b128"])
def test_conv_wgrad_halo(gpu_device, shape):
    """Halo-patch WGRAD (3x3 / stride 1, one input window per 128-pixel block for all nine taps; the automatic
    choice for these shapes) vs torch, and vs the generic split-K WGRAD (an explicit split count) on the same
    inputs."""
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device, seed=23)
    wr_ = wb.clone().requires_grad_(True)
    ref = F.conv2d(x, wr_, stride=1, padding=1)
    gy = torch.randn_like(ref).bfloat16().float()
    ref.backward(gy)
    dyn = _nhwc(gy).bfloat16()
    shp = (xn.shape, O, R, R, st, pad, Cw)
    ws = torch.full((conv.wgrad_ws_floats(*shp),), float("nan"), device=gpu_device)
    dw = conv.conv2d_wgrad(xn, dyn, 3, 3, 1, 1, Cw=Cw, ws=ws)
    ws0 = torch.full((2 * O * 9 * xn.shape[-1],), float("nan"), device=gpu_device)
    dw0 = conv.conv2d_wgrad(xn, dyn, 3, 3, 1, 1, Cw=Cw, ws=ws0, splits=2)
    torch.cuda.synchronize()
    assert not torch.isnan(dw).any()
    assert _rel(dw, wr_.grad) < 1e-2
    assert _rel(dw, dw0) < 1e-3


# DGRAD epilogue with a second incoming grad and the producer BN's backward sums (conv_igemm.hip BnSums):
# single-pass tap kernel, split-K combine, and the four stride-2 sub-pixel phases
FUSE_SHAPES = [(8, 16, 16, 64, 64, 3, 1, 1), (128, 32, 32, 64, 64, 3, 1, 1), (128, 8, 8, 256, 256, 3, 1, 1),
               (128, 4, 4, 512, 512, 3, 1, 1), (16, 16, 16, 64, 128, 3, 2, 1), (16, 8, 8, 128, 256, 1, 1, 0),
               # stride-1 DGRAD on conv_tap<GEN> (O % 64 != 0): GoogLeNet's narrow branches
               (16, 32, 32, 16, 32, 3, 1, 1), (16, 16, 16, 96, 48, 1, 1, 0)]


@pytest.mark.parametrize("shape", FUSE_SHAPES, ids=[str(s) for s in FUSE_SHAPES])
@pytest.mark.parametrize("relu,proj,zmask", [(True, False, False), (False, True, False), (False, False, True)],
                         ids=["ymask", "proj", "zmask"])
def test_conv_dgrad_fused_bn_sums(gpu_device, shape, relu, proj, zmask):
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device, seed=31)
    C = xn.shape[-1]
    P = (H + 2 * pad - R) // st + 1
    g = torch.Generator(device="cpu").manual_seed(5)
    dyn = torch.randn(N, P, P, O, generator=g).to(gpu_device).bfloat16()
    add = torch.randn(N, H, W, C, generator=g).to(gpu_device).bfloat16()
    z = torch.randn(N, H, W, C, generator=g).to(gpu_device).bfloat16()
    y = torch.relu(torch.randn(N, H, W, C, generator=g)).to(gpu_device).bfloat16() if relu else None
    zb = torch.randn(N, H, W, C, generator=g).to(gpu_device).bfloat16() if proj else None
    mean, inv = torch.randn(C, device=gpu_device) * 0.1, torch.rand(C, device=gpu_device) + 0.5
    meanb, invb = torch.randn(C, device=gpu_device) * 0.1, torch.rand(C, device=gpu_device) + 0.5
    wpk = conv.pack_weight(w)
    wd = torch.empty(conv.dgrad_image_numel(w.shape, C), dtype=torch.bfloat16, device=gpu_device)
    conv.dgrad_pack_weights([(w, wd, st, pad, C)])
    shp = (xn.shape, O, R, R, st, pad, Cw)
    assert conv.dgrad_fusable(*shp)
    wsp = torch.empty(max(conv.fd_ws_floats(*shp), 1), device=gpu_device)
    reps = 4
    rep = torch.zeros(reps, 3, C, dtype=torch.float64, device=gpu_device)
    bs = dict(rep=rep, reps=reps, z=z, y=y, mean=mean, inv=inv)
    if proj:
        bs.update(zb=zb, meanb=meanb, invb=invb)
    msc = torch.stack([torch.rand(C, device=gpu_device) + 0.5, torch.randn(C, device=gpu_device) * 0.5])
    if zmask:   # ReLU mask derived from z with the forward's scale / shift (y never re-read)
        bs.update(msc=msc)
    plain = conv.conv2d_dgrad(dyn, wpk, xn.shape, st, pad, Cw=Cw, ws=wsp, wd=wd)
    out = torch.full_like(plain, float("nan"))
    conv.conv2d_dgrad(dyn, wpk, xn.shape, st, pad, Cw=Cw, out=out, ws=wsp, wd=wd, add=add, bn_sums=bs)
    torch.cuda.synchronize()
    # out = bf16(dgrad + add): one or two bf16 roundings of the same sum
    ref = plain.float() + add.float()
    assert float((out.float() - ref).abs().max()) <= 2 * float(ref.abs().max()) * 2 ** -8
    # the sums are of the stored bf16 output (what bn_bwd's apply pass re-reads)
    gm = out.double().reshape(-1, C)
    if relu:
        gm = torch.where(y.double().reshape(-1, C) > 0, gm, torch.zeros_like(gm))
    if zmask:
        m = torch.addcmul(msc[1], z.float().reshape(-1, C), msc[0]) > 0
        gm = torch.where(m, gm, torch.zeros_like(gm))
    s0 = gm.sum(0)
    s1 = (gm * ((z.double().reshape(-1, C) - mean.double()) * inv.double())).sum(0)
    got = rep.sum(0)
    scale = gm.abs().sum(0) + 1.0
    assert float(((got[0] - s0).abs() / scale).max()) < 1e-5
    assert float(((got[1] - s1).abs() / (scale * 4)).max()) < 1e-5
    if proj:
        s2 = (gm * ((zb.double().reshape(-1, C) - meanb.double()) * invb.double())).sum(0)
        assert float(((got[2] - s2).abs() / (scale * 4)).max()) < 1e-5
    else:
        assert float(got[2].abs().max()) == 0.0


def test_bn_bwd_presummed_matches_reduce(gpu_device):
    """bn_bwd's apply pass on epilogue-summed replicas == the reduce + apply pair (chained mode)."""
    M, C = 4096, 128
    g = torch.Generator(device="cpu").manual_seed(9)
    dy = torch.randn(M, C, generator=g).to(gpu_device).bfloat16()
    z = torch.randn(M, C, generator=g).to(gpu_device).bfloat16()
    y = torch.relu(torch.randn(M, C, generator=g)).to(gpu_device).bfloat16()
    gamma = torch.rand(C, device=gpu_device) + 0.5
    mean, inv = torch.randn(C, device=gpu_device) * 0.1, torch.rand(C, device=gpu_device) + 0.5
    reps = cnn.bn_bwd_chain_floats(C) // (3 * C)
    outs = []
    for pres in (False, True):
        rep = torch.zeros(reps, 3, C, dtype=torch.float64, device=gpu_device)
        if pres:   # what the DGRAD epilogue adds: the sums of masked dy over the rows, split over replicas
            gm = torch.where(y.float() > 0, dy.float(), torch.zeros_like(dy.float())).double()
            rep[0, 0] = gm.sum(0)
            rep[0, 1] = (gm * ((z.double() - mean.double()) * inv.double())).sum(0)
        a = cnn.bn_desc(gamma=gamma, smean=mean, sinv=inv)
        dg, db = torch.empty(C, device=gpu_device), torch.empty(C, device=gpu_device)
        dz = torch.empty(M, C, dtype=torch.bfloat16, device=gpu_device)
        red = torch.zeros(3, C, dtype=torch.float64, device=gpu_device)
        cnn.bn_bwd(dy, z, a, dg, db, dz, red, y=y, ws=rep.view(-1), chained=True, presummed=pres)
        torch.cuda.synchronize()
        outs.append((dz.float(), dg, db))
    (dz0, dg0, db0), (dz1, dg1, db1) = outs
    assert _rel(dg1, dg0) < 1e-5 and _rel(db1, db0) < 1e-5
    assert _rel(dz1, dz0) < 1e-2


@pytest.mark.parametrize("shape", [(16, 16, 16, 64, 1), (128, 32, 32, 64, 1), (32, 8, 8, 96, 2), (8, 4, 4, 1024, 1)],
                         ids=["c64", "c64_b128", "c96_s2", "c1024"])
def test_dwconv_dgrad_fused_bn_sums(gpu_device, shape):
    """Depthwise DGRAD with the producer BN's backward sums (MobileNet block boundaries)."""
    N, H, W, C, st = shape
    g = torch.Generator(device="cpu").manual_seed(13)
    P = (H + 2 - 3) // st + 1
    dy = torch.randn(N, P, P, C, generator=g).to(gpu_device).bfloat16()
    w = (torch.randn(C, 1, 3, 3, generator=g) / 3).to(gpu_device)
    z = torch.randn(N, H, W, C, generator=g).to(gpu_device).bfloat16()
    y = torch.relu(torch.randn(N, H, W, C, generator=g)).to(gpu_device).bfloat16()
    mean, inv = torch.randn(C, device=gpu_device) * 0.1, torch.rand(C, device=gpu_device) + 0.5
    plain = conv.dwconv_dgrad(dy, w, (N, H, W, C), st, 1)
    rep = torch.zeros(4, 3, C, dtype=torch.float64, device=gpu_device)
    out = conv.dwconv_dgrad(dy, w, (N, H, W, C), st, 1, bn_sums=dict(rep=rep, reps=4, z=z, y=y, mean=mean, inv=inv))
    torch.cuda.synchronize()
    assert torch.equal(out, plain)
    gm = out.double().reshape(-1, C)
    gm = torch.where(y.double().reshape(-1, C) > 0, gm, torch.zeros_like(gm))
    s0 = gm.sum(0)
    s1 = (gm * ((z.double().reshape(-1, C) - mean.double()) * inv.double())).sum(0)
    got = rep.sum(0)
    scale = gm.abs().sum(0) + 1.0
    assert float(((got[0] - s0).abs() / scale).max()) < 1e-5
    assert float(((got[1] - s1).abs() / (scale * 4)).max()) < 1e-5


@pytest.mark.parametrize("shape", [(4, 16, 16, 64, 128, 1, 2, 0), (128, 8, 8, 256, 512, 1, 2, 0)])
def test_conv_dgrad_1x1_stride2_zeroes_tapless_parities(gpu_device, shape):
    """1x1 / stride 2: three of the four dX parities get no tap.  They ride in the one tap-phases launch as K = 0
    phases that write zeros -- every element of a NaN-filled output must be overwritten."""
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device, seed=23)
    xr = x.clone().requires_grad_(True)
    out = F.conv2d(xr, wb, stride=st, padding=pad)
    gy = torch.randn_like(out).bfloat16().float()
    out.backward(gy)
    C = xn.shape[-1]
    wd = torch.empty(conv.dgrad_image_numel(w.shape, C), dtype=torch.bfloat16, device=gpu_device)
    conv.dgrad_pack_weights([(w, wd, st, pad, C)])
    shp = (xn.shape, O, R, R, st, pad, Cw)
    wsp = torch.empty(max(conv.fd_ws_floats(*shp), 1), device=gpu_device)
    dx = torch.full_like(xn, float("nan"))
    conv.conv2d_dgrad(_nhwc(gy).bfloat16(), conv.pack_weight(w), xn.shape, st, pad, Cw=Cw, out=dx, ws=wsp, wd=wd)
    torch.cuda.synchronize()
    assert not torch.isnan(dx.float()).any()
    assert torch.equal(dx[:, 1::2].float(), torch.zeros_like(dx[:, 1::2].float()))
    assert _rel(dx[..., :Cw].float(), _nhwc(xr.grad)) < 1e-2


@pytest.mark.parametrize("shape", [(3, 7, 5, 3, 32, 3, 1, 1), (2, 32, 32, 3, 64, 3, 1, 1), (5, 9, 9, 3, 64, 3, 1, 1),
                                   (500, 32, 32, 3, 32, 3, 1, 1)],
                         ids=["odd_o32", "b2_o64", "b5_9x9", "eval500_o32"])
def test_conv_stem_kernel(gpu_device, shape):
    """The network-input conv kernel (conv_stem_kernel: C = 8 padded, 3x3 / stride 1, O = 32 | 64) vs torch fp32,
    with BatchNorm statistics of bf16(y) - shift (M not a multiple of 16 included), and without statistics."""
    N, H, W, Cw, O, R, st, pad = shape
    x, w, wb, xn = _make(shape, gpu_device, seed=31)
    wr = conv.pack_weight(w)
    shift = (torch.randn(O, device=gpu_device) * 0.1)
    rep = conv.stats_buffer(O, gpu_device)
    y = conv.conv2d_fwd(xn, wr, st, pad, Cw=Cw, stats=rep, shift=shift)
    y2 = conv.conv2d_fwd(xn, wr, st, pad, Cw=Cw)
    ref = F.conv2d(x, wb, stride=st, padding=pad)
    torch.cuda.synchronize()
    assert _rel(y.float(), _nhwc(ref)) < 1e-2
    assert torch.equal(y, y2)
    d = y.float().reshape(-1, O) - shift
    stats = conv.stats_total(rep)
    assert torch.allclose(stats[0], d.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(stats[1], (d * d).sum(0), rtol=1e-3, atol=1e-2)


def test_conv_fwd_tap_gen_sweep(gpu_device):
    """conv_tap<GEN> (C % 8, several taps per 64-deep K step) against fp32 over random shapes: channel counts
    off the 64 grid (DenseNet / DPN / GoogLeNet widths), 1x1 / 3x3 / 5x5, stride 1 / 2, partial row tiles, K
    shorter than one step, and long K (split-K)."""
    g = torch.Generator().manual_seed(77)
    shapes = [(2, 4, 4, 16, 16, 1, 1, 0), (2, 5, 5, 24, 8, 1, 2, 0), (4, 8, 8, 304, 96, 1, 1, 0),
              (4, 8, 8, 336, 200, 1, 2, 0), (3, 16, 16, 96, 96, 3, 2, 1), (2, 7, 9, 40, 72, 3, 1, 1),
              (16, 4, 4, 600, 256, 1, 1, 0), (8, 4, 4, 648, 512, 3, 1, 1), (2, 11, 11, 56, 24, 5, 1, 2)]
    for _ in range(8):
        R = [1, 3, 5][int(torch.randint(0, 3, (1,), generator=g))]
        C = 8 * int(torch.randint(2, 90 if R < 5 else 40, (1,), generator=g))    # (weight pack: C * R * S rows)
        if C % 64 == 0:
            C += 8
        O = 8 * int(torch.randint(1, 40, (1,), generator=g))
        st = int(torch.randint(1, 3, (1,), generator=g))
        H = int(torch.randint(3, 17, (1,), generator=g))
        shapes.append((int(torch.randint(1, 6, (1,), generator=g)), H, H, C, O, R, st, R // 2))
    for shape in shapes:
        N, H, W, Cw, O, R, st, pad = shape
        x, w, wb, xn = _make(shape, gpu_device, seed=5)
        wr = conv.pack_weight(w)
        rep = conv.stats_buffer(O, gpu_device)
        y = conv.conv2d_fwd(xn, wr, st, pad, Cw=Cw, stats=rep, ws=conv.wgrad_workspace(gpu_device, 1 << 24))
        ref = F.conv2d(x, wb, stride=st, padding=pad)
        torch.cuda.synchronize()
        assert _rel(y.float(), _nhwc(ref)) < 1e-2, shape
        stats = conv.stats_total(rep)
        yb = y.float()
        assert torch.allclose(stats[0], yb.sum((0, 1, 2)), rtol=1e-3, atol=5e-2), shape
