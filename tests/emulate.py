"""PyTorch emulation of the fedmi CNN kernels (tests and debugging only).

Every function here has the signature and buffer semantics of its native
counterpart in :mod:`fedmi.ops.conv` / :mod:`fedmi.ops.cnn` (NHWC bf16
activations, fp32 stats, outputs written in place) but computes with plain
torch ops, so the native engines' *wiring* — which buffer feeds which launch,
residual fan-in, BN branch pairing, running-stat updates — can be verified on
a CPU-only host.  :func:`emulated` swaps them in for the duration of a
``with`` block.  Never used on a GPU run: the native paths fail loudly when
the extension is missing instead of falling back here.
"""
from __future__ import annotations

import contextlib
from typing import Optional

import torch
import torch.nn.functional as F

from fedmi.ops import cnn, conv

_BF = torch.bfloat16


def _nchw(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 3, 1, 2).float()


def _nhwc_into(out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    out.copy_(t.permute(0, 2, 3, 1).to(out.dtype))
    return out


# packed image -> fp32 master it was packed from: the emulated convolutions use
# the master weights, so an fp32-activation run is exact up to fp32 rounding
_MASTER: dict = {}


@torch.no_grad()
def pack_weight(w, c_pad=None, out=None):
    O, Cw, R, S = w.shape
    C = c_pad or conv.pad8(Cw)
    img = torch.zeros(O, R, S, C, dtype=_BF, device=w.device)
    img[..., :Cw] = w.permute(0, 2, 3, 1).to(_BF)
    if out is None:
        out = img
    else:
        out.copy_(img)
    _MASTER[out.data_ptr()] = w
    return out


def pack_weights(items):
    for w, out in items:
        pack_weight(w, out.shape[3], out=out)


def fd_ws_floats(*a, **k):
    return 0


def dgrad_pack_weights(items):
    pass


class SgdPack:
    """conv.SgdPack under emulation: the torch SGD update of the flat master, then the forward images."""

    def __init__(self, params, grad, mom, convs):
        self.p, self.g, self.m = params, grad, mom
        self.convs = [(w, wr) for w, wr, *_rest in convs]
        self.n_convs = len(self.convs)

    @torch.no_grad()
    def step(self, lr, momentum, weight_decay, dampening=0.0, nesterov=False, first=False):
        d = self.g + weight_decay * self.p
        if momentum != 0:
            self.m.copy_(d if first else momentum * self.m + (1 - dampening) * d)
            d = d + momentum * self.m if nesterov else self.m
        self.p.sub_(lr * d)
        for w, wr in self.convs:
            if wr is not None:
                pack_weight(w, wr.shape[3], out=wr)


def _w_from_img(wr: torch.Tensor, Cw: Optional[int]) -> torch.Tensor:
    m = _MASTER.get(wr.data_ptr())
    w = m.float() if m is not None and m.shape[2:] == wr.shape[1:3] else wr.permute(0, 3, 1, 2).float()
    return w if Cw is None else w[:, :Cw]


def _stats_add(stats, y_bf16_nhwc, shift=None):
    if stats is not None:
        v = y_bf16_nhwc.float().reshape(-1, y_bf16_nhwc.shape[-1])
        if shift is not None:
            v = v - shift
        rep0 = stats.view(conv.STAT_REP, 2, -1)[0]     # replica 0 (the native kernels spread over all)
        rep0[0] += v.sum(0)
        rep0[1] += (v * v).sum(0)


@torch.no_grad()
def conv2d_fwd(x, wrsc, stride, pad, Cw=None, stats=None, out=None, shift=None, ws=None, res=None):
    Cw = Cw or x.shape[3]
    y = F.conv2d(_nchw(x)[:, :Cw], _w_from_img(wrsc, Cw), stride=stride, padding=pad)
    if res is not None:
        y = y + _nchw(res)
    if out is None:
        out = torch.empty(y.shape[0], y.shape[2], y.shape[3], y.shape[1], dtype=_BF, device=x.device)
    _nhwc_into(out, y)
    _stats_add(stats, out, shift)
    return out


@torch.no_grad()
def conv2d_dgrad(dy, wrsc, x_shape, stride, pad, Cw=None, out=None, ws=None, wd=None, accumulate=False, add=None,
                 bn_sums=None):
    """``bn_sums``: the kernel adds the producer BN's backward sums into its replicas; the emulated
    bn_bwd recomputes them from dya either way, so only the schedule (``add``) matters here."""
    N, H, W, C = x_shape
    Cw = Cw or C
    O, R, S = wrsc.shape[0], wrsc.shape[1], wrsc.shape[2]
    if (add is not None or bn_sums is not None) and not dgrad_fusable(x_shape, O, R, S, stride, pad, Cw,
                                                                     wd is not None):
        raise ValueError("conv2d_dgrad: add / bn_sums need a fusable shape")
    dx = torch.nn.grad.conv2d_input((N, Cw, H, W), _w_from_img(wrsc, Cw), _nchw(dy), stride=stride, padding=pad)
    full = torch.zeros(N, C, H, W, device=dy.device)
    full[:, :Cw] = dx
    if out is None:
        out = torch.empty(*x_shape, dtype=_BF, device=dy.device)
    if accumulate:
        full = full + _nchw(out)
    if add is not None:
        full = _nchw(_nhwc_into(torch.empty_like(out), full)).float() + _nchw(add).float()
    return _nhwc_into(out, full)


def dgrad_fusable(x_shape, O, R, S, stride, pad, Cw=None, has_wd=True):
    """Mirror of conv_igemm.hip conv_dgrad_fusable: tap path (a DGRAD image; O % 64, or stride 1 and O % 8 from 16
    channels), no empty phase."""
    if not has_wd or not (O % 64 == 0 or (stride == 1 and O % 8 == 0 and O >= 16)):
        return False
    if stride == 1:
        return True
    H, W = x_shape[1], x_shape[2]
    for ph in range(2):
        for pw in range(2):
            r0, s0 = (ph + pad) & 1, (pw + pad) & 1
            nr, ns = max(0, (R - r0 + 1) // 2), max(0, (S - s0 + 1) // 2)
            if (H - ph + 1) // 2 > 0 and (W - pw + 1) // 2 > 0 and nr * ns == 0:
                return False
    return True


@torch.no_grad()
def conv2d_wgrad(x, dy, R, S, stride, pad, Cw=None, out=None, accumulate=False, splits=0, ws=None, deferred=None,
                 lib_gemm=True):
    # deferred: the emulation reduces immediately (nothing to append)
    Cw = Cw or x.shape[3]
    O = dy.shape[3]
    dw = torch.nn.grad.conv2d_weight(_nchw(x)[:, :Cw], (O, Cw, R, S), _nchw(dy), stride=stride, padding=pad)
    if out is None:
        return dw
    if accumulate:
        out += dw
    else:
        out.copy_(dw)
    return out


def wgrad_ws_floats(*a, **k):
    return 1


def wgrad_reduce_multi(items, device):
    assert not items, "the emulated WGRAD reduces immediately"


def dwconv_fwd(x, w, stride, pad, stats=None, out=None, shift=None):
    C = x.shape[3]
    y = F.conv2d(_nchw(x), w.float(), stride=stride, padding=pad, groups=C)
    if out is None:
        out = torch.empty(y.shape[0], y.shape[2], y.shape[3], C, dtype=_BF, device=x.device)
    _nhwc_into(out, y)
    _stats_add(stats, out, shift)
    return out


@torch.no_grad()
def dwconv_dgrad(dy, w, x_shape, stride, pad, out=None, bn_sums=None):
    N, H, W, C = x_shape
    dx = torch.nn.grad.conv2d_input((N, C, H, W), w.float(), _nchw(dy), stride=stride, padding=pad, groups=C)
    if out is None:
        out = torch.empty(*x_shape, dtype=_BF, device=dy.device)
    return _nhwc_into(out, dx)


@torch.no_grad()
def dwconv_wgrad(x, dy, R, stride, pad, out=None, accumulate=False, ws=None, deferred=None):
    C = x.shape[3]
    dw = torch.nn.grad.conv2d_weight(_nchw(x), (C, 1, R, R), _nchw(dy), stride=stride, padding=pad,
                                     groups=C)
    if out is None:
        return dw
    if accumulate:
        out += dw
    else:
        out.copy_(dw)
    return out


def dwconv_ws_floats(*a, **k):
    return 1


@torch.no_grad()
def prep_input(images_u8, base, nb, augment, seed, round_ctr, out=None, dbase=None):
    import numpy as np

    from fedmi.engine.data import augment_normalize

    b = base + (int(dbase.view(-1)[0]) if dbase is not None else 0)
    gidx = np.arange(b, b + nb) if augment else None
    x = augment_normalize(images_u8[b:b + nb], gidx, seed, int(round_ctr.view(-1)[0]))
    full = torch.zeros(nb, 8, 32, 32, device=images_u8.device)
    full[:, :3] = x
    if out is None:
        out = torch.empty(nb, 32, 32, 8, dtype=_BF, device=images_u8.device)
    return _nhwc_into(out, full)


@torch.no_grad()
def sched_next(sched, counter, cur, zero=None):
    if zero is not None:
        zero.zero_()
    i = int(counter.view(-1)[0])
    cur.view(-1)[0] = sched.view(-1)[i]
    counter.view(-1)[0] = i + 1


def _coeffs(p: "cnn.BNParams", M: int, train: bool, eps: float, mom: float):
    if train:
        tot = conv.stats_total(p.stats).float()
        ms = tot[0] / M
        var = torch.clamp(tot[1] / M - ms * ms, min=0.0)
        mean = ms + (p.shift if p.shift is not None else 0.0)
        inv = torch.rsqrt(var + eps)
        p.smean.copy_(mean)
        p.sinv.copy_(inv)
        if p.rmean is not None:
            p.rmean.mul_(1 - mom).add_(mom * (mean + (p.cbias if p.cbias is not None else 0.0)))
            p.rvar.mul_(1 - mom).add_(mom * var * M / max(M - 1, 1))
        if p.nbt is not None:
            p.nbt += 1
    else:
        mean, inv = p.rmean - (p.cbias if p.cbias is not None else 0.0), torch.rsqrt(p.rvar + eps)
    sc = p.gamma * inv
    return sc, p.beta - mean * sc


@torch.no_grad()
def bn_apply(z, a, y, train, relu, z2=None, b=None, res=None, eps=1e-5, momentum=0.1, co_out=None):
    C = z.shape[-1]
    M = z.numel() // C
    sc, sh = _coeffs(a, M, train, eps, momentum)
    if co_out is not None:
        co_out[0].copy_(sc)
        co_out[1].copy_(sh)
    v = z.float().reshape(M, C) * sc + sh
    if b is not None:
        sc2, sh2 = _coeffs(b, M, train, eps, momentum)
        v = v + z2.float().reshape(M, C) * sc2 + sh2
    elif res is not None:
        v = v + res.float().reshape(M, C)
    if relu:
        v = torch.relu(v)
    y.copy_(v.reshape(y.shape).to(y.dtype))
    return y


@torch.no_grad()
def maxpool3(x, stride, out=None, idx=None):
    y, ind = F.max_pool2d(_nchw(x), 3, stride, 1, return_indices=True)
    if out is None:
        out = torch.empty(y.shape[0], y.shape[2], y.shape[3], y.shape[1], dtype=x.dtype, device=x.device)
    _nhwc_into(out, y)
    # emulation keeps the input itself (not the kernel's tap bytes): overlapping windows need autograd's sum
    return out, x


def maxpool3_bwd(dy, idx, x_shape, stride, out=None, accumulate=False):
    xr = _nchw(idx).requires_grad_(True)
    with torch.enable_grad():
        F.max_pool2d(xr, 3, stride, 1).backward(_nchw(dy))
    g = xr.grad
    if out is None:
        out = torch.empty(*x_shape, dtype=dy.dtype, device=dy.device)
    if accumulate:
        g = g + _nchw(out)
    return _nhwc_into(out, g)


@torch.no_grad()
def maxpool2(x, out=None):
    y = F.max_pool2d(_nchw(x), 2, 2)
    if out is None:
        out = torch.empty(y.shape[0], y.shape[2], y.shape[3], y.shape[1], dtype=x.dtype, device=x.device)
    return _nhwc_into(out, y)


def maxpool2_bwd(x, dy, out=None):
    xr = _nchw(x).requires_grad_(True)
    with torch.enable_grad():
        F.max_pool2d(xr, 2, 2).backward(_nchw(dy))
    if out is None:
        out = torch.empty_like(x)
    return _nhwc_into(out, xr.grad)


@torch.no_grad()
def bn_bwd(dya, za, a, dgamma_a, dbeta_a, dza, red, dyb=None, y=None, zb=None, b=None, dgamma_b=None,
           dbeta_b=None, dzb=None, gout=None, ws=None, dadd=None, chained=False, mask_bn=None, presummed=False):
    if presummed and (dyb is not None or not chained):
        raise ValueError("bn_bwd: presummed covers one incoming grad, chained replicas")
    C = za.shape[-1]
    M = za.numel() // C
    g = dya.float().reshape(M, C)
    if dyb is not None:
        g = g + dyb.float().reshape(M, C)
    if y is not None:
        g = torch.where(y.float().reshape(M, C) > 0, g, torch.zeros_like(g))
    elif mask_bn is not None:
        g = torch.where(za.float().reshape(M, C) * mask_bn[0] + mask_bn[1] > 0, g, torch.zeros_like(g))
    if gout is not None:
        gout.copy_(g.reshape(gout.shape).to(gout.dtype))
    sg = g.sum(0)
    for z, p, dg, db, dz in ((za, a, dgamma_a, dbeta_a, dza), (zb, b, dgamma_b, dbeta_b, dzb)):
        if z is None:
            continue
        xhat = (z.float().reshape(M, C) - p.smean) * p.sinv
        sgx = (g * xhat).sum(0)
        dg.copy_(sgx)
        db.copy_(sg)
        if p.shift is not None:
            p.shift.copy_(p.smean)
        d = p.gamma * p.sinv * (g - sg / M - xhat * sgx / M)
        if dadd is not None and z is za:
            d = d + dadd.float().reshape(M, C)
        dz.copy_(d.reshape(dz.shape).to(dz.dtype))


def bn_bwd_ws_floats(M, C):
    return 0


def bn_bwd_chain_floats(C):
    return 12 * C    # a replica slice exists (the engine then takes the chained / presummed schedule)


@torch.no_grad()
def head(y, labels, base, W, b, stats, train, pooled=None, dlog=None, dy=None, dW=None, db=None, dbase=None,
         zero=None, lossv=None):
    if zero is not None:
        zero.zero_()
    N, H, Wd, C = y.shape
    base = base + (int(dbase.view(-1)[0]) if dbase is not None else 0)
    lab = labels[base:base + N].long()
    pl = y.float().reshape(N, H * Wd, C).mean(1)
    logits = pl @ W.t() + b
    lse = torch.logsumexp(logits, 1)
    stats[0] += float((lse - logits.gather(1, lab[:, None])[:, 0]).sum())
    iv = stats.view(torch.int32)
    iv[1] += int((logits.argmax(1) == lab).sum())
    iv[2] += N
    if not train:
        return
    dl = (torch.softmax(logits, 1) - F.one_hot(lab, W.shape[0]).float()) / N
    pooled.copy_(pl)
    dlog.copy_(dl)
    dW.copy_(dl.t() @ pl)
    db.copy_(dl.sum(0))
    dp = (dl @ W) / (H * Wd)
    dy.copy_(dp[:, None, None, :].expand(N, H, Wd, C).to(dy.dtype))


class _NativeStub:
    """Stands in for the extension module under emulation: only flat SGD is needed."""

    @staticmethod
    def sgd_flat(st, p, g, buf, n, lr, m, wd, damp, nesterov, first):
        raise RuntimeError("emulated engine: use the torch update path")


@contextlib.contextmanager
def emulated():
    """Swap fedmi.ops kernels (and native.require) for their torch emulations."""
    from fedmi import native

    saved = []

    def swap(mod, name, fn):
        saved.append((mod, name, getattr(mod, name)))
        setattr(mod, name, fn)

    for name in ("pack_weight", "pack_weights", "SgdPack", "fd_ws_floats", "dgrad_pack_weights", "conv2d_fwd", "conv2d_dgrad", "dgrad_fusable", "conv2d_wgrad", "wgrad_ws_floats", "wgrad_reduce_multi", "dwconv_fwd",
                 "dwconv_dgrad", "dwconv_wgrad", "dwconv_ws_floats"):
        swap(conv, name, globals()[name])
    for name in ("prep_input", "sched_next", "bn_apply", "bn_bwd", "bn_bwd_ws_floats", "bn_bwd_chain_floats", "head", "maxpool2",
                 "maxpool2_bwd", "maxpool3", "maxpool3_bwd"):
        swap(cnn, name, globals()[name])
    swap(native, "require", lambda: _NativeStub())
    swap(native, "stream_handle", lambda device=None: 0)
    try:
        yield
    finally:
        for mod, name, fn in reversed(saved):
            setattr(mod, name, fn)
