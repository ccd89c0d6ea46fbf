"""BatchNorm / classifier-head / input-prep kernels (csrc/kernels/cnn_ops.hip).

All activations NHWC bf16 flattened to ``[M, C]`` rows (M = N*H*W).
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import native


def _p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def prep_input(images_u8: torch.Tensor, base: int, nb: int, augment: bool, seed: int, round_ctr: torch.Tensor,
               out: Optional[torch.Tensor] = None, dbase: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 [Ntot, 3, 32, 32] rows [base, base+nb) -> augmented, normalised bf16 [nb, 32, 32, 8].

    ``dbase`` (int32 device scalar) is added to ``base`` on the device (graph replays); the caller
    guarantees base + dbase + nb <= Ntot in that case (schedules are validated when set).
    """
    if images_u8.dtype != torch.uint8 or tuple(images_u8.shape[1:]) != (3, 32, 32):
        raise ValueError("prep_input: expects uint8 [N, 3, 32, 32]")
    if dbase is None and (base < 0 or base + nb > images_u8.shape[0]):
        raise ValueError("prep_input: batch out of range")
    if out is None:
        out = torch.empty(nb, 32, 32, 8, dtype=torch.bfloat16, device=images_u8.device)
    native.require().prep_input(native.stream_handle(images_u8.device), images_u8.data_ptr(), base, _p(dbase), nb,
                                int(augment), seed & 0xFFFFFFFF, round_ctr.data_ptr(), out.data_ptr())
    return out


def sched_next(sched: torch.Tensor, counter: torch.Tensor, cur: torch.Tensor, zero: torch.Tensor = None) -> None:
    """cur = sched[counter++] on the device; ``zero`` (fp64, contiguous, 16-B aligned): zeroed in the same launch."""
    if zero is not None:
        assert zero.dtype == torch.float64 and zero.is_contiguous() and zero.data_ptr() % 16 == 0
    native.require().sched_next(native.stream_handle(sched.device), sched.data_ptr(), counter.data_ptr(),
                                cur.data_ptr(), zero.data_ptr() if zero is not None else 0,
                                zero.numel() if zero is not None else 0)


class BNParams:
    """One BatchNorm2d's device tensors (train-time batch stats + params + running/saved stats)."""

    __slots__ = ("stats", "gamma", "beta", "rmean", "rvar", "nbt", "smean", "sinv", "shift", "cbias")

    def __init__(self, stats=None, gamma=None, beta=None, rmean=None, rvar=None, nbt=None, smean=None, sinv=None,
                 shift=None, cbias=None):
        self.stats, self.gamma, self.beta = stats, gamma, beta
        self.rmean, self.rvar, self.nbt = rmean, rvar, nbt
        self.smean, self.sinv = smean, sinv
        # ``stats`` hold sums of (z - shift); bn_bwd stores this step's batch mean into ``shift``
        self.shift = shift
        # bias of the producing conv (VGG / GoogLeNet convs have one), kept OUT of z: a train-mode BN
        # is invariant to it (its gradient is exactly 0); it only enters running_mean and eval
        self.cbias = cbias

    def ptrs(self) -> dict:
        return {k: _p(getattr(self, k)) for k in self.__slots__}


def row_stride(t: torch.Tensor) -> int:
    """Row stride (elements) of an NHWC / [M, C] tensor that may be a channel slice of a wider buffer
    (a branch's output inside a concatenated tensor); rows must be evenly spaced, channels unit-stride."""
    if t.is_contiguous():
        return int(t.shape[-1])
    st, sh = t.stride(), t.shape
    if st[-1] != 1:
        raise ValueError("channel dimension must be unit-stride")
    ld = st[-2]
    for d in range(t.dim() - 2):
        if st[d] != st[d + 1] * sh[d + 1]:
            raise ValueError("rows of a channel-slice view must be evenly spaced")
    if ld % 8 or t.data_ptr() % 16:
        raise ValueError("channel-slice views need 16-byte aligned rows (offset and stride % 8)")
    return int(ld)


def bn_desc(stats=None, gamma=None, beta=None, rmean=None, rvar=None, nbt=None, smean=None, sinv=None,
            shift=None, cbias=None) -> BNParams:
    return BNParams(stats, gamma, beta, rmean, rvar, nbt, smean, sinv, shift, cbias)


def maxpool3(x: torch.Tensor, stride: int, out: Optional[torch.Tensor] = None,
             idx: Optional[torch.Tensor] = None):
    """MaxPool2d(3, stride, padding=1) of NHWC bf16 ``x``; returns (y, idx) with idx the uint8 window argmax."""
    N, H, W, C = x.shape
    P, Q = (H - 1) // stride + 1, (W - 1) // stride + 1
    if out is None:
        out = torch.empty(N, P, Q, C, dtype=x.dtype, device=x.device)
    if idx is None:
        idx = torch.empty(N, P, Q, C, dtype=torch.uint8, device=x.device)
    native.require().maxpool3(native.stream_handle(x.device), x.data_ptr(), out.data_ptr(), idx.data_ptr(), N, H, W, C,
                              int(stride))
    return out, idx


def maxpool3_bwd(dy: torch.Tensor, idx: torch.Tensor, x_shape, stride: int, out: Optional[torch.Tensor] = None,
                 accumulate: bool = False) -> torch.Tensor:
    """dx of :func:`maxpool3` (gather over the covering windows); ``accumulate``: dx += instead of =."""
    N, H, W, C = (int(v) for v in x_shape)
    if out is None:
        out = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
    native.require().maxpool3_bwd(native.stream_handle(dy.device), dy.data_ptr(), idx.data_ptr(), out.data_ptr(), N, H,
                                  W, C, int(stride), int(accumulate))
    return out


def maxpool2(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """MaxPool2d(2, 2) of NHWC bf16 ``x`` [N, H, W, C] (H, W even, C % 8 == 0)."""
    N, H, W, C = x.shape
    if out is None:
        out = torch.empty(N, H // 2, W // 2, C, dtype=x.dtype, device=x.device)
    native.require().maxpool2(native.stream_handle(x.device), x.data_ptr(), out.data_ptr(), N, H, W, C)
    return out


def maxpool2_bwd(x: torch.Tensor, dy: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dx of MaxPool2d(2, 2): dy routed to each window's first maximum of ``x``, 0 elsewhere."""
    N, H, W, C = x.shape
    if tuple(dy.shape) != (N, H // 2, W // 2, C):
        raise ValueError("maxpool2_bwd: dy shape mismatch")
    if out is None:
        out = torch.empty_like(x)
    native.require().maxpool2_bwd(native.stream_handle(x.device), x.data_ptr(), dy.data_ptr(), out.data_ptr(),
                                  N, H, W, C)
    return out


def bn_apply(z: torch.Tensor, a: BNParams, y: torch.Tensor, train: bool, relu: bool,
             z2: Optional[torch.Tensor] = None, b: Optional[BNParams] = None, res: Optional[torch.Tensor] = None,
             eps: float = 1e-5, momentum: float = 0.1, co_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = act(BN_a(z) [+ res | + BN_b(z2)]) over [M, C] rows; train mode commits running stats.
    ``co_out``: float32 [2, C] <- BN_a's scale / shift as applied (a backward that derives the ReLU mask
    from z instead of re-reading y)."""
    C = z.shape[-1]
    M = z.numel() // C
    if co_out is not None and (co_out.dtype != torch.float32 or co_out.numel() < 2 * C):
        raise ValueError("bn_apply: co_out must be float32 [2, C]")
    native.require().bn_apply(native.stream_handle(z.device), z.data_ptr(), a.ptrs(), _p(z2),
                              b.ptrs() if b is not None else None, _p(res), y.data_ptr(), M, C, eps, momentum,
                              int(train), int(relu), row_stride(y), _p(co_out))
    return y


def bn_bwd(dya: torch.Tensor, za: torch.Tensor, a: BNParams, dgamma_a: torch.Tensor, dbeta_a: torch.Tensor,
           dza: torch.Tensor, red: torch.Tensor, dyb: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None,
           zb: Optional[torch.Tensor] = None, b: Optional[BNParams] = None, dgamma_b=None, dbeta_b=None, dzb=None,
           gout: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
           dadd: Optional[torch.Tensor] = None, chained: bool = False,
           mask_bn: Optional[torch.Tensor] = None, presummed: bool = False) -> None:
    """BatchNorm backward through an optional ReLU mask (``y``: forward output) for one or two BN
    branches sharing the incoming grad g = dya (+ dyb).  Writes dz for each branch, dgamma/dbeta,
    and optionally g itself (``gout``, the identity-shortcut grad).  ``red``: [3, C] fp64 channel
    sums.  With ``ws`` (>= :func:`bn_bwd_ws_floats` fp64, ZERO before first use; every call leaves it
    zero) the sums go through replicated atomics + a finalize and ``red`` needs no init; without,
    they are atomics straight into ``red``, which must be ZERO.  ``chained``: ``ws`` is this BN's own
    replica buffer (>= :func:`bn_bwd_chain_floats`, ZERO on entry -- the engine's head launch clears
    the arena every step); no finalize launch, the apply kernel reads the replicas.  ``mask_bn``
    ([2, C] scale / shift, with ``y`` None): the ReLU mask is relu(za * scale + shift) > 0 -- for a BN
    whose output was never materialised (its consumer applied it on load).  ``presummed`` (chained): the
    DGRAD that wrote ``dya`` already added the channel sums into ``ws`` (:func:`conv.conv2d_dgrad`
    ``bn_sums``): only the apply pass runs."""
    C = za.shape[-1]
    M = za.numel() // C
    if red.numel() < 3 * C or red.dtype != torch.float64:
        raise ValueError("bn_bwd: red must be fp64 with >= 3*C elements")
    if ws is not None and ws.dtype != torch.float64:
        raise ValueError("bn_bwd: ws must be fp64")
    d = dict(dya=_p(dya), dyb=_p(dyb), y=_p(y), za=_p(za), meanA=_p(a.smean), invA=_p(a.sinv), gammaA=_p(a.gamma),
             dgammaA=_p(dgamma_a), dbetaA=_p(dbeta_a), dza=_p(dza), gout=_p(gout), shiftA=_p(a.shift),
             dadd=_p(dadd), msc=_p(mask_bn))
    if zb is not None:
        d.update(zb=_p(zb), meanB=_p(b.smean), invB=_p(b.sinv), gammaB=_p(b.gamma), dgammaB=_p(dgamma_b),
                 dbetaB=_p(dbeta_b), dzb=_p(dzb), shiftB=_p(b.shift))
    ldd = row_stride(dya)
    if dyb is not None and row_stride(dyb) != ldd:
        raise ValueError("bn_bwd: dya and dyb must share a row stride")
    native.require().bn_bwd(native.stream_handle(red.device), d, red.data_ptr(), M, C,
                            ws.data_ptr() if ws is not None else 0, ws.numel() if ws is not None else 0,
                            ldd, row_stride(y) if y is not None else C, int(chained), int(presummed))


def bn_bwd_chain_floats(C: int) -> int:
    """fp64 replica elements one BN needs in chained mode."""
    return 3 * int(C) * int(native.require().bn_bwd_chain_reps(int(C)))


def bn_bwd_ws_floats(M: int, C: int) -> int:
    return int(native.require().bn_bwd_ws_floats(int(M), int(C)))


def head(y: torch.Tensor, labels: torch.Tensor, base: int, W: torch.Tensor, b: torch.Tensor, stats: torch.Tensor,
         train: bool, pooled=None, dlog=None, dy=None, dW=None, db=None, dbase=None,
         zero: Optional[torch.Tensor] = None, lossv: Optional[torch.Tensor] = None) -> None:
    """Global avgpool + linear + CE (+ correct count) of y [N,H,W,C] bf16; with ``train`` also the CE
    gradient into ``dy`` and the linear layer's ``dW`` / ``db``.  ``lossv``: [N] fp32 scratch for the
    per-sample losses, summed into ``stats`` in sample order (bit-reproducible; no float atomics)."""
    N, H, Wd, C = y.shape
    J = W.shape[0]
    if lossv is None:
        lossv = torch.empty(N, dtype=torch.float32, device=y.device)
    native.require().head(native.stream_handle(y.device), y.data_ptr(), labels.data_ptr(), base, _p(dbase), N,
                          H * Wd, C, J,
                          W.data_ptr(), b.data_ptr(), _p(pooled), _p(dlog), _p(dy), stats.data_ptr(), _p(dW), _p(db),
                          int(train), _p(zero), zero.numel() * zero.element_size() // 4 if zero is not None else 0,
                          lossv.data_ptr())
