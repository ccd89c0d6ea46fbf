"""A native aten backend for the zoo families without a whole-network engine.

:class:`NativeMode` is a ``TorchDispatchMode``: while it is active, every aten op
of a training step that launches device work -- forward AND the backward ops
autograd generates -- is executed by fedmi's HIP kernels instead of ATen/MIOpen/
rocBLAS:

* convolutions: the MFMA implicit-GEMM kernels (``conv_igemm.hip``: forward,
  data gradient, weight gradient) for dense convs with 8-aligned channels, the
  depthwise kernels (``dwconv.hip``), one MFMA GEMM per group for few wide groups
  (ResNeXt), and a direct VALU kernel (``zoo_ops.hip``) for every other grouped /
  odd-width conv (DPN, ShuffleNet, RegNet, the 3-channel stems);
* BatchNorm (train + eval, running statistics), elementwise / activation ops with
  broadcasting, channel concat / slice gradients, spatial reductions (SE gates,
  bias gradients), avg / max pooling, the classifier GEMMs, log-softmax + NLL,
  dropout / drop-connect masks (a counter-based RNG keyed by a device step counter,
  so a replayed HIP graph draws fresh masks) -- all in ``zoo_ops.hip``.

Metadata ops (views, expand, transpose, detach, empty) pass through: they launch
nothing.  Output shapes / strides / dtypes follow ATen's own meta functions where
the operands share a dtype, so layouts (channels-last activations) are preserved.
Ops without a native implementation are counted in :attr:`NativeMode.fallbacks`
(and raise with ``strict=True``): the GPU tests assert that a training step of
every hybrid family needs none.

Reference ops: the union of SURVEY.md §2.4(d) (convolution(+backward), addmm/mm,
native_batch_norm(+backward), relu / threshold_backward, avg_pool2d, cat,
max_pool2d_with_indices, sigmoid, mul, mean, slice_backward, bernoulli_, ...).
"""
from __future__ import annotations

import collections
import sys
import os
import math
from typing import Optional

import torch
import torch.nn.functional as F
from torch.overrides import TorchFunctionMode
from torch.utils._python_dispatch import TorchDispatchMode

from .. import native
from . import conv as CV

aten = torch.ops.aten

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.int64: 2}

# elementwise op codes (zoo_ops.hip EwOp)
EW_COPY, EW_ADD, EW_MUL, EW_MULS, EW_RELU, EW_THR_BWD, EW_SIGMOID, EW_SIG_BWD, EW_FILL, EW_FMA = range(10)
EW_BNB, EW_BERN, EW_SUB, EW_DIV, EW_ADDS, EW_FMA_RELU, EW_BNB_THR = 11, 12, 13, 14, 15, 16, 17
EW_FMA_ADD, EW_FMA_ADD_RELU, EW_BNB_ADD, EW_BNB_THR_ADD = 18, 19, 20, 21
# an impl returns ATEN when the op is legitimately ATen's (host copies, scalar reads): not a fallback
ATEN = object()
RD_SUM, RD_SUMSQ_SHIFT, RD_DOT_SHIFT, RD_DOT_R = 0, 1, 2, 3


def _nat():
    return native.require()


def _st(dev) -> int:
    return native.stream_handle(dev)


def zd(t: Optional[torch.Tensor]):
    """(ptr, dtype code, sizes, strides) descriptor of a CUDA tensor (None passes through)."""
    if t is None:
        return None
    if t.dtype not in _DT:
        raise TypeError(f"native_mode: unsupported dtype {t.dtype}")
    if t.numel() >= (1 << 31):
        raise ValueError("native_mode: tensors must have < 2^31 elements")
    if t.dim() == 0:
        return (t.data_ptr(), _DT[t.dtype], [1], [1])
    return (t.data_ptr(), _DT[t.dtype], list(t.shape), list(t.stride()))


def _bcast(t: torch.Tensor, shape) -> torch.Tensor:
    if tuple(t.shape) == tuple(shape):
        return t
    return t.expand(shape) if t.dim() == len(shape) else t.reshape((1,) * (len(shape) - t.dim()) + tuple(t.shape)).expand(shape)


def coalesce(shape, strides):
    """Merge the dims of an iteration space shared by several operands (``strides``: one stride list per
    operand, operand 0 decides the order): size-1 dims drop, dims are ordered by operand 0's strides and
    neighbours that are contiguous in EVERY operand merge -- a channels-last activation with a
    per-channel operand becomes [N*H*W, C], a pure elementwise op one flat dim."""
    dims = [d for d in range(len(shape)) if shape[d] != 1]
    if not dims:
        return [1], [[0] for _ in strides]
    dims.sort(key=lambda d: -abs(strides[0][d]))
    nshape = [shape[dims[0]]]
    nstr = [[s[dims[0]]] for s in strides]
    for d in dims[1:]:
        if all(ns[-1] == s[d] * shape[d] for ns, s in zip(nstr, strides)):
            nshape[-1] *= shape[d]
            for ns, s in zip(nstr, strides):
                ns[-1] = s[d]
        else:
            nshape.append(shape[d])
            for ns, s in zip(nstr, strides):
                ns.append(s[d])
    return nshape, nstr


def ew(out: torch.Tensor, ins, op: int, s0: float = 0.0, s1: float = 0.0, seed: int = 0, ctr=None) -> torch.Tensor:
    """out[...] = op(ins...) with broadcasting of every input to out's shape."""
    if out.numel() == 0:
        return out
    if out.numel() >= (1 << 31):
        raise ValueError("native_mode: tensors must have < 2^31 elements")
    shape = list(out.shape) if out.dim() else [1]
    o = out if out.dim() else out.view(1)
    ts = [_bcast(t if t.dim() else t.view(1), shape) for t in ins]
    for t in ts:
        if t.dtype not in _DT:
            raise TypeError(f"native_mode: unsupported dtype {t.dtype}")
    if op == EW_BERN:
        # the counter-based mask is a function of the logical element index: keep the logical order
        nshape, nstr = shape, [list(o.stride())] + [list(t.stride()) for t in ts]
    else:
        nshape, nstr = coalesce(shape, [list(o.stride())] + [list(t.stride()) for t in ts])
    allt = [o] + ts
    vw, vmask = 8, -1
    if op != EW_BERN:
        for vw in (8, 4):
            vmask = _vec_mask(nshape, nstr, allt, vw)
            if vmask >= 0:
                break
    if vmask >= 0:
        nshape = nshape[:-1] + [nshape[-1] // vw]
        nstr = [st[:-1] + [st[-1] * vw] for st in nstr]
    if NativeMode.current is not None and NativeMode.current.diag:   # passes per op code, and which miss the vector launch
        NativeMode.current.ew_ops[(NativeMode.current._func_name(), op)] += 1
        if vmask < 0:
            NativeMode.current.scalar_ew[(op, tuple(out.shape), tuple(out.stride()),
                                          tuple(tuple(t.stride()) for t in ts))] += 1
    descs = [(t.data_ptr(), _DT[t.dtype], nshape, st) for t, st in zip(allt, nstr)]
    _nat().z_ew(_st(out.device), descs[0], descs[1:], op, float(s0), float(s1), int(seed) & 0xFFFFFFFF,
                0 if ctr is None else ctr.data_ptr(), vmask, vw)
    return out


def _vec_mask(shape, strides, ts, vw: int = 8) -> int:
    """Bit k (input k) set if that operand is contiguous over groups of ``vw`` innermost elements, bit
    clear = a broadcast operand; -1 = the vector launch does not apply (odd sizes, misalignment,
    int64, an output that is not unit-stride innermost, fp32 with vw 4 below 16-byte alignment)."""
    if shape[-1] % vw:
        return -1
    mask = 0
    for k, (t, st) in enumerate(zip(ts, strides)):
        inner = st[-1]
        if inner == 0 and k > 0:
            continue
        align = 16 if (t.dtype == torch.float32 or vw == 8) else 8
        if inner != 1 or t.dtype == torch.int64 or t.data_ptr() % align or any(v % vw for v in st[:-1]):
            return -1
        if k > 0:
            mask |= 1 << (k - 1)
    return mask


def fill_(t: torch.Tensor, v: float) -> torch.Tensor:
    return ew(t, [], EW_FILL, v)


def _scalar(x) -> Optional[float]:
    """A Python number or a CPU 0-dim 'wrapped number' tensor -> float; a device tensor -> None."""
    if isinstance(x, (int, float, bool)):
        return float(x)
    if isinstance(x, torch.Tensor) and x.dim() == 0 and not x.is_cuda:
        return float(x.item())
    return None


def _meta(t):
    if isinstance(t, torch.Tensor):
        return torch.empty_strided(t.shape, t.stride(), dtype=t.dtype, device="meta")
    if isinstance(t, (list, tuple)):
        return type(t)(_meta(v) for v in t)
    return t


def _alloc_like_meta(func, args, kwargs, dev):
    """Run ATen's meta function for the output metadata, allocate real (uninitialised) outputs."""
    m = func(*_meta(args), **{k: _meta(v) for k, v in kwargs.items()})
    if isinstance(m, torch.Tensor):
        return torch.empty_strided(m.shape, m.stride(), dtype=m.dtype, device=dev)
    return type(m)(torch.empty_strided(t.shape, t.stride(), dtype=t.dtype, device=dev) for t in m)


def _dev(*ts):
    for t in ts:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            return t.device
        if isinstance(t, (list, tuple)):
            d = _dev(*t)
            if d is not None:
                return d
    return None


def _rowmajor_out(out: torch.Tensor) -> bool:
    """out's elements sit at their row-major index (size-1 dims ignored): a reduction can store into it by the
    accumulator index."""
    if out.dtype not in (torch.float32, torch.bfloat16):
        return False
    expect = 1
    for d in range(out.dim() - 1, -1, -1):
        if out.shape[d] == 1:
            continue
        if out.stride(d) != expect:
            return False
        expect *= out.shape[d]
    return True


def reduce_sum(a: torch.Tensor, dims, acc: Optional[torch.Tensor], op: int = RD_SUM, b: Optional[torch.Tensor] = None,
               shift: Optional[torch.Tensor] = None, acc2: Optional[torch.Tensor] = None,
               out: Optional[torch.Tensor] = None, scale: float = 1.0) -> None:
    """acc (fp32, ZEROED, one entry per kept element in order) += sum over ``dims`` of f(a[, b]); or, with
    ``out`` (RD_SUM, :func:`_rowmajor_out`), out = scale * sum stored directly (no zeroed accumulator, no copy:
    the bias gradients, spatial means of SE gates, sums of autograd's broadcast backward)."""
    dims = sorted(d % a.dim() for d in dims)
    kept = [d for d in range(a.dim()) if d not in dims]
    ops = [a] if b is None else [a, b]

    def space(ds, order_by_acc):
        if not ds:
            return [1], [[0] for _ in ops]
        shp = [a.shape[d] for d in ds]
        strs = [[t.stride(d) for d in ds] for t in ops]
        if order_by_acc:
            # kept dims: the accumulator index is row-major over them -- merge only, never reorder
            acc_str = [1] * len(ds)
            for j in range(len(ds) - 2, -1, -1):
                acc_str[j] = acc_str[j + 1] * shp[j + 1]
            ns, nst = coalesce(shp, [acc_str] + strs)
            return ns, nst[1:]
        return coalesce(shp, strs)

    oshape, ostr = space(kept, True)
    ishape, istr = space(dims, False)
    if op != RD_DOT_R and _rows_ok(oshape, ostr, ishape, istr, ops):
        # channels-last moments / bias gradients: [M, C] rows, 16-byte channel vectors, deterministic
        C, M = oshape[0], ishape[0]
        nat = _nat()
        part = torch.empty(int(nat.z_reduce_rows_ws_floats(M, C)), dtype=torch.float32, device=a.device)
        nat.z_reduce_rows(_st(a.device), a.data_ptr(), _DT[a.dtype], istr[0][0],
                          b.data_ptr() if b is not None else 0, _DT[b.dtype] if b is not None else 0,
                          istr[1][0] if b is not None else 0, shift.data_ptr() if shift is not None else 0, C, M, op,
                          part.data_ptr(), part.numel(), acc.data_ptr() if acc is not None else 0,
                          acc2.data_ptr() if acc2 is not None else 0, out.data_ptr() if out is not None else 0,
                          _DT[out.dtype] if out is not None else 0, float(scale))
        return
    outer = (0, 0, oshape, ostr[0])
    inner = (0, 0, ishape, istr[0])
    outer_b = (0, 0, oshape, ostr[1]) if b is not None else None
    inner_b = (0, 0, ishape, istr[1]) if b is not None else None
    nat = _nat()
    # split partials summed in a fixed order afterwards (no float atomics: bitwise-reproducible steps)
    nws = int(nat.z_reduce_ws_floats(math.prod(oshape), math.prod(ishape)))
    part = torch.empty(max(nws, 1), dtype=torch.float32, device=a.device)
    nat.z_reduce(_st(a.device), outer, inner, outer_b, inner_b, a.data_ptr(), _DT[a.dtype],
                 b.data_ptr() if b is not None else 0, _DT[b.dtype] if b is not None else 0,
                 shift.data_ptr() if shift is not None else 0, acc.data_ptr() if acc is not None else 0,
                 acc2.data_ptr() if acc2 is not None else 0, op, part.data_ptr(), nws,
                 out.data_ptr() if out is not None else 0, _DT[out.dtype] if out is not None else 0, float(scale))


def _rows_ok(oshape, ostr, ishape, istr, ops) -> bool:
    if len(oshape) != 1 or len(ishape) != 1 or oshape[0] % 4 or ishape[0] < 1:
        return False
    vw = 8 if oshape[0] % 8 == 0 else 4
    for t, os_, is_ in zip(ops, ostr, istr):
        align = 16 if (t.dtype == torch.float32 or vw == 8) else 8
        if os_[0] != 1 or is_[0] % vw or t.dtype not in (torch.float32, torch.bfloat16) or t.data_ptr() % align:
            return False
    return True


# ---------------------------------------------------------------------------- op impls
_IMPL = {}


def impl(*ops):
    def deco(fn):
        for o in ops:
            _IMPL[o] = fn
        return fn
    return deco


# ---- elementwise ---------------------------------------------------------------
@impl(aten.add.Tensor, aten.sub.Tensor)
def _add(func, self, other, alpha=1):
    mode = NativeMode.current
    if func is aten.add.Tensor and alpha == 1 and mode is not None and mode._pend_bn is not None:
        pend = mode._pend_bn
        res = _bn_add_partner(pend, (self, other))
        if res is not None:         # BN(x) + shortcut joins the pending apply pass; the BN output stays deferred
            out = torch.empty_like(pend.out)
            mode._pend_bn = _PendingBN(out, pend.x, pend.scale, pend.shift, res)
            mode._defer(pend.out, pend.materialize)
            mode.fused["bn+add"] += 1
            return out
    pair = _sb_pair(mode, (self, other), {"alpha": alpha}) if func is aten.add.Tensor else None
    if pair is not None:            # slice_backward(g1, [0, a)) + slice_backward(g2, [a, n)): two copies
        lo, hi = pair
        out = torch.empty_like(lo.out)
        ew(out.narrow(lo.dim, lo.start, lo.end - lo.start), [lo.grad], EW_COPY)
        ew(out.narrow(hi.dim, hi.start, hi.end - hi.start), [hi.grad], EW_COPY)
        mode.fused["slice_bwd+add"] += 1
        return out
    if func is aten.add.Tensor and mode is not None and mode._pend_bnb is not None:
        o = _bnb_add_partner(mode._pend_bnb, (self, other), {"alpha": alpha})
        if o is not None:           # BN-backward gradient + the other incoming gradient: one pass
            pend, mode._pend_bnb = mode._pend_bnb, None
            out = _alloc_like_meta(func, (self, other), {"alpha": alpha}, self.device)
            pend.add(out, o)
            mode._defer(pend.out, pend.materialize)
            mode.fused["bn_bwd+grad_add"] += 1
            return out
    sign = -1.0 if func is aten.sub.Tensor else 1.0
    s = _scalar(other)
    if s is not None:
        return ew(torch.empty_like(self), [self], EW_ADDS, sign * alpha * s)
    out = _alloc_like_meta(func, (self, other), {"alpha": alpha}, self.device)
    return ew(out, [self, other], EW_ADD, sign * alpha)


@impl(aten.add_.Tensor, aten.sub_.Tensor)
def _add_(func, self, other, alpha=1):
    sign = -1.0 if func is aten.sub_.Tensor else 1.0
    s = _scalar(other)
    mode = NativeMode.current
    if (s is not None and mode is not None and mode.fuse and func is aten.add_.Tensor and sign * alpha * s == 1.0
            and self.dtype == torch.int64 and self.numel() == 1):
        # BatchNorm's num_batches_tracked += 1 (torch.nn.modules.batchnorm, right before the batch_norm call): the
        # BN forward's finalizing workgroup bumps it, so it costs no launch of its own
        mode._flush_ctr()
        mode._pend_ctr = self
        mode.fused["bn_counter"] += 1
        return self
    if func is aten.add_.Tensor and mode is not None and mode._pend_bnb is not None:
        o = _bnb_add_partner(mode._pend_bnb, (self, other), {"alpha": alpha})
        if o is not None:           # in-place accumulation into either operand: one pass
            pend, mode._pend_bnb = mode._pend_bnb, None
            pend.add(self, o)
            if o is self:
                mode._defer(pend.out, pend.materialize)
            mode.fused["bn_bwd+grad_add"] += 1
            return self
    if s is not None:
        return ew(self, [self], EW_ADDS, sign * alpha * s)
    return ew(self, [self, other], EW_ADD, sign * alpha)


class _PendingMul:
    """a * b (same shapes) not computed yet: if the next op sums it over some dims (autograd's backward of a
    broadcast multiply -- the SE gate's gradient), the product is folded into that reduction (RD_DOT_SHIFT,
    no shift) and never stored; any other op materialises it."""
    __slots__ = ("out", "a", "b")

    def __init__(self, out, a, b):
        self.out, self.a, self.b = out, a, b

    def materialize(self):
        ew(self.out, [self.a, self.b], EW_MUL)


@impl(aten.mul.Tensor)
def _mul(func, self, other):
    s = _scalar(other)
    if s is not None:
        return ew(torch.empty_like(self), [self], EW_MULS, s)
    s = _scalar(self)
    if s is not None:
        return ew(torch.empty_like(other), [other], EW_MULS, s)
    out = _alloc_like_meta(func, (self, other), {}, _dev(self, other))
    mode = NativeMode.current
    if (mode is not None and mode.fuse and self.shape == other.shape == out.shape and self.dtype == other.dtype
            and out.dim() >= 2):
        mode._pend_mul = _PendingMul(out, self, other)
        return out
    return ew(out, [self, other], EW_MUL)


@impl(aten.mul_.Tensor)
def _mul_(func, self, other):
    s = _scalar(other)
    if s is not None:
        return ew(self, [self], EW_MULS, s)
    return ew(self, [self, other], EW_MUL)


@impl(aten.mul.Scalar)
def _mul_s(func, self, other):
    return ew(torch.empty_like(self), [self], EW_MULS, float(other))


@impl(aten.div.Scalar)
def _div_s(func, self, other):
    return ew(torch.empty_like(self), [self], EW_MULS, 1.0 / float(other))


@impl(aten.div_.Scalar)
def _div_s_(func, self, other):
    return ew(self, [self], EW_MULS, 1.0 / float(other))


@impl(aten.div.Tensor)
def _div_t(func, self, other):
    s = _scalar(other)
    if s is not None:
        return ew(torch.empty_like(self), [self], EW_MULS, 1.0 / s)
    out = _alloc_like_meta(func, (self, other), {}, _dev(self, other))
    return ew(out, [self, other], EW_DIV)


@impl(aten.relu.default)
def _relu(func, self):
    pend = _mode_pending_bn(self)
    if pend is not None:            # relu(BN(x) [+ res]) in ONE pass; the pre-ReLU tensor stays deferred (dead)
        out = torch.empty_like(self)
        pend.relu(out)
        NativeMode.current._defer(self, pend.materialize)
        NativeMode.current.fused["bn+relu" if pend.res is None else "bn+add+relu"] += 1
        return out
    return ew(torch.empty_like(self), [self], EW_RELU)


@impl(aten.relu_.default)
def _relu_(func, self):
    pend = _mode_pending_bn(self)
    if pend is not None:            # the pending output is overwritten by its ReLU: one pass, nothing deferred
        NativeMode.current.fused["bn+relu_" if pend.res is None else "bn+add+relu_"] += 1
        return pend.relu(self)
    return ew(self, [self], EW_RELU)


class _PendingBNB:
    """A BatchNorm input gradient whose apply pass has not run: when autograd next sums it with the tensor's
    other incoming gradient (DenseNet: the concat's slice; residual nets: the shortcut), the sum joins the
    pass (EW_BNB[_THR]_ADD, the gradient rounded as the unfused pair stores it); any other op materialises it."""
    __slots__ = ("out", "ins", "thr")

    def __init__(self, out, ins, thr):
        self.out, self.ins, self.thr = out, ins, thr

    def materialize(self):
        ew(self.out, self.ins, EW_BNB_THR if len(self.ins) == 6 else EW_BNB, self.thr)

    def add(self, out, other):
        rnd = 1.0 if self.out.dtype == torch.bfloat16 else 0.0
        return ew(out, self.ins + [other], EW_BNB_THR_ADD if len(self.ins) == 6 else EW_BNB_ADD, self.thr, rnd)


def _bnb_add_partner(pend, args, kwargs=None):
    """The other operand of ``add(a, b)`` / ``a.add_(b)`` when one operand is the pending BN-backward gradient
    (plain sum, same shape and dtype); else None."""
    if pend is None or len(args) != 2 or (kwargs and kwargs.get("alpha", 1) != 1):
        return None
    a, b = args
    if not (isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor)):
        return None
    o = b if _same(a, pend.out) else a if _same(b, pend.out) else None
    if o is None or o.shape != pend.out.shape or o.dtype != pend.out.dtype:
        return None
    return o


class _PendingThr:
    """threshold_backward(grad, relu_out) not yet computed: its consumer (BN backward) masks on the fly."""
    __slots__ = ("out", "grad", "relu_out", "thr")

    def __init__(self, out, grad, relu_out, thr):
        self.out, self.grad, self.relu_out, self.thr = out, grad, relu_out, thr

    def materialize(self):
        ew(self.out, [self.grad, self.relu_out], EW_THR_BWD, self.thr)


@impl(aten.threshold_backward.default)
def _thr_bwd(func, grad_output, self, threshold):
    out = _alloc_like_meta(func, (grad_output, self, threshold), {}, grad_output.device)
    mode = NativeMode.current
    if (mode is not None and mode.fuse and _cl_rows(grad_output) and _cl_rows(self) and _cl_rows(out)
            and grad_output.shape == self.shape):
        mode._pend_thr = _PendingThr(out, grad_output, self, float(threshold))
        return out
    return ew(out, [grad_output, self], EW_THR_BWD, float(threshold))


@impl(aten.sigmoid.default)
def _sigmoid(func, self):
    return ew(torch.empty_like(self), [self], EW_SIGMOID)


@impl(aten.sigmoid_backward.default)
def _sigmoid_bwd(func, grad_output, output):
    out = _alloc_like_meta(func, (grad_output, output), {}, grad_output.device)
    return ew(out, [grad_output, output], EW_SIG_BWD)


@impl(aten._to_copy.default)
def _to_copy(func, self, **kw):
    dev = kw.get("device")
    if not self.is_cuda or (dev is not None and torch.device(dev).type != "cuda"):
        return ATEN                                   # host copies stay ATen (not a device kernel)
    mkw = {k: v for k, v in kw.items() if k not in ("device", "pin_memory", "non_blocking")}
    out = _alloc_like_meta(func, (self,), mkw, self.device)
    return ew(out, [self], EW_COPY)


@impl(aten.clone.default)
def _clone(func, self, memory_format=None):
    out = _alloc_like_meta(func, (self,), {"memory_format": memory_format} if memory_format else {}, self.device)
    return ew(out, [self], EW_COPY)


@impl(aten.copy_.default)
def _copy_(func, self, src, non_blocking=False):
    if not (src.is_cuda and self.is_cuda):
        return ATEN                                   # H2D / D2H transfer, not a compute kernel
    return ew(self, [src], EW_COPY)


@impl(aten.ones_like.default, aten.zeros_like.default)
def _fill_like(func, self, **kw):
    out = _alloc_like_meta(func, (self,), kw, self.device)
    return fill_(out, 1.0 if func is aten.ones_like.default else 0.0)


@impl(aten.new_zeros.default, aten.new_ones.default)
def _new_fill(func, self, size, **kw):
    out = _alloc_like_meta(func, (self, size), kw, self.device)
    return fill_(out, 1.0 if func is aten.new_ones.default else 0.0)


@impl(aten.fill_.Scalar)
def _fill_s(func, self, value):
    return fill_(self, float(value))


@impl(aten.zero_.default)
def _zero_(func, self):
    return fill_(self, 0.0)


# ---- concat / slicing -------------------------------------------------------------
class _CatBuf:
    """A reverse-filled concat buffer: NHWC [N, H, W, K], channels [front, K) live.  ``cat([y, x], 1)`` with x
    the live tail writes y in front of it and returns the longer tail -- x is never copied again (DenseNet's
    growing feature map, /root/reference/src/models/densenet.py:20-24: the reference copies the whole map per
    layer)."""
    __slots__ = ("buf", "front", "head")

    def __init__(self, buf, front, head):
        self.buf, self.front, self.head = buf, front, head

    def tail(self):
        return _nchw(self.buf[..., self.front:])


def _cat_chain(mode, y: torch.Tensor, x: torch.Tensor):
    """``cat([y, x], 1)`` of 4-D activations through a concat buffer, or None (the plain copy path).

    A chain is a run of such cats, each taking the previous one's output as x.  The first block that runs a
    chain only learns its final width (``mode._cat_plan``, keyed by the head cat's shapes); from then on the
    head cat allocates a buffer of that width and every later cat of the chain copies only its y.  Aliasing is
    safe because nothing writes a cat output in place (:meth:`NativeMode.__torch_dispatch__` refuses in-place
    ops on a buffer) and each buffer hands out only ever-longer tails."""
    if x.dim() != 4 or y.dim() != 4 or x.dtype != y.dtype or x.shape[0] != y.shape[0] or x.shape[2:] != y.shape[2:]:
        return None
    N, Cy, H, W = y.shape
    Cx = x.shape[1]
    ent = mode._catbufs.get(x.untyped_storage().data_ptr())
    if ent is not None and ent.front >= Cy and _same(x, ent.tail()):
        ew(_nchw(ent.buf[..., ent.front - Cy:ent.front]), [y], EW_COPY)
        ent.front -= Cy
        out = ent.tail()
        mode._cat_plan[ent.head] = max(mode._cat_plan.get(ent.head, 0), Cx + Cy)
        mode.fused["cat_in_place"] += 1
        return out
    head = mode._cat_src.get((x.data_ptr(), tuple(x.shape)))
    if head is not None:                 # learning: x is an earlier cat's output, the chain grows
        mode._cat_plan[head] = max(mode._cat_plan.get(head, 0), Cx + Cy)
        return None
    head = (N, H, W, Cx, Cy, x.dtype)
    K = CV.pad8(mode._cat_plan.get(head, 0))
    if K <= Cx + Cy:
        return head                      # not (yet) known to be a chain head: plain copy, remember the head
    buf = torch.empty(N, H, W, K, dtype=x.dtype, device=x.device)
    ent = _CatBuf(buf, K - Cx, head)
    ew(ent.tail(), [x], EW_COPY)
    ew(_nchw(buf[..., ent.front - Cy:ent.front]), [y], EW_COPY)
    ent.front -= Cy
    mode._catbufs[buf.untyped_storage().data_ptr()] = ent
    return ent.tail()


@impl(aten.cat.default)
def _cat(func, tensors, dim=0):
    tensors = [t for t in tensors if t.numel() > 0 or t.dim() > 1]
    mode = NativeMode.current
    head = None
    if mode is not None and mode.fuse and len(tensors) == 2 and tensors[0].dim() == 4 and dim % 4 == 1:
        r = _cat_chain(mode, tensors[0], tensors[1])
        if isinstance(r, torch.Tensor):
            return r
        head = r
    out = _alloc_like_meta(func, (tensors,), {"dim": dim}, _dev(tensors))
    if (out.dim() == 4 and dim % 4 == 1 and not out.is_contiguous(memory_format=torch.channels_last)
            and all(t.dim() == 4 and t.stride(1) == 1 for t in tensors)):
        # channel slices of channels-last activations (DPN's dual path) make ATen's meta pick NCHW: keep the
        # activations channels-last (vector copies here, no layout transposes in the next conv)
        out = torch.empty(out.shape, dtype=out.dtype, device=out.device, memory_format=torch.channels_last)
    d = dim % out.dim()
    off = 0
    for t in tensors:
        if t.numel():
            ew(out.narrow(d, off, t.shape[d]), [t], EW_COPY)
        off += t.shape[d] if t.dim() else 0
    if mode is not None and mode.fuse and len(tensors) == 2 and tensors[0].dim() == 4 and dim % 4 == 1:
        x = tensors[1]
        src = mode._cat_src.get((x.data_ptr(), tuple(x.shape)))
        mode._cat_src[(out.data_ptr(), tuple(out.shape))] = src if src is not None else head
    return out


class _PendingSliceBwd:
    """slice_backward not computed yet (zeros + the gradient in its slice): autograd's sum of two of them that
    tile the sliced dim (DPN's dual path: y[:, :d] and y[:, d:]) becomes two copies into one tensor -- no zero
    fills, no add pass; any other read materialises it."""
    __slots__ = ("out", "grad", "dim", "start", "end", "done")

    def __init__(self, out, grad, dim, start, end):
        self.out, self.grad, self.dim, self.start, self.end = out, grad, dim, start, end
        self.done = False

    def materialize(self):
        self.done = True
        fill_(self.out, 0.0)
        ew(self.out.narrow(self.dim, self.start, self.end - self.start), [self.grad], EW_COPY)


def _sb_pair(mode, args, kwargs=None):
    """The two pending slice_backwards an ``add(a, b)`` sums when their slices tile the dim exactly, else None."""
    if mode is None or not mode._pend_sb or len(args) != 2 or (kwargs and kwargs.get("alpha", 1) != 1):
        return None
    a, b = args
    if not (isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor)) or not (a.is_cuda and b.is_cuda):
        return None
    pa = mode._pend_sb.get(a.untyped_storage().data_ptr())
    pb = mode._pend_sb.get(b.untyped_storage().data_ptr())
    if (pa is None or pb is None or pa is pb or pa.done or pb.done or not (_same(a, pa.out) and _same(b, pb.out))
            or pa.dim != pb.dim):
        return None
    lo, hi = (pa, pb) if pa.start <= pb.start else (pb, pa)
    if lo.start != 0 or lo.end != hi.start or hi.end != pa.out.shape[pa.dim]:
        return None
    return lo, hi


@impl(aten.slice_backward.default)
def _slice_bwd(func, grad_output, input_sizes, dim, start, end, step):
    out = _alloc_like_meta(func, (grad_output, input_sizes, dim, start, end, step), {}, grad_output.device)
    if out.dim() == 4 and grad_output.stride(1) == 1 and not out.is_contiguous(memory_format=torch.channels_last):
        # the meta function allocates NCHW zeros: keep a channels-last gradient channels-last (DPN's dual-path
        # slices would otherwise turn every upstream BN backward and conv gradient into layout transposes)
        out = torch.empty(out.shape, dtype=out.dtype, device=out.device, memory_format=torch.channels_last)
    d = dim % out.dim()
    lo = max(0, min(start, out.shape[d])) if start is not None else 0
    hi = max(lo, min(end, out.shape[d])) if end is not None else out.shape[d]
    mode = NativeMode.current
    if mode is not None and mode.fuse and step == 1 and hi - lo == grad_output.shape[d]:
        pend = _PendingSliceBwd(out, grad_output, d, lo, hi)
        mode._pend_sb[out.untyped_storage().data_ptr()] = pend
        mode._defer(out, pend.materialize)
        return out
    fill_(out, 0.0)
    ew(aten.slice.Tensor(out, dim, start, end, step), [grad_output], EW_COPY)
    return out


# ---- reductions ----------------------------------------------------------------
def _sum_like(func, self, dim, keepdim, dtype, scale_by_count: bool):
    dims = list(range(self.dim())) if dim is None or len(dim) == 0 else [d % self.dim() for d in dim]
    kw = {"keepdim": keepdim}
    if dtype is not None:
        kw["dtype"] = dtype
    out = _alloc_like_meta(func, (self, dim), kw, self.device)
    cnt = 1
    for d in dims:
        cnt *= self.shape[d]
    mode = NativeMode.current
    pend = mode._pend_mul if mode is not None else None
    if pend is not None and _same(self, pend.out):
        mode._pend_mul = None
        kept = [d for d in range(self.dim()) if d not in dims and self.shape[d] > 1]
        # per-(sample, channel) sums (SE gates): the generic reduction, which the unfused sum takes too
        if out.numel() and _rowmajor_out(out) and len(kept) >= 2:   # sum(a * b): one dot reduction, the product never stored
            # bf16 operands: each product rounded as the unfused multiply stores it (fused == unfused, bitwise)
            rd = RD_DOT_R if pend.out.dtype == torch.bfloat16 else RD_DOT_SHIFT
            reduce_sum(pend.a, dims, None, rd, b=pend.b, out=out,
                       scale=1.0 / max(cnt, 1) if scale_by_count else 1.0)
            mode._defer(pend.out, pend.materialize)
            mode.fused["mul+sum"] += 1
            return out
        pend.materialize()
    if out.numel() and _rowmajor_out(out):
        reduce_sum(self, dims, None, out=out, scale=1.0 / max(cnt, 1) if scale_by_count else 1.0)
        return out
    acc = torch.empty(out.shape, dtype=torch.float32, device=self.device)
    fill_(acc, 0.0)
    reduce_sum(self, dims, acc)
    if scale_by_count:
        return ew(out, [acc], EW_MULS, 1.0 / max(cnt, 1))
    return ew(out, [acc], EW_COPY)


@impl(aten.sum.dim_IntList)
def _sum(func, self, dim, keepdim=False, dtype=None):
    return _sum_like(func, self, dim, keepdim, dtype, False)


@impl(aten.mean.dim)
def _mean(func, self, dim, keepdim=False, dtype=None):
    return _sum_like(func, self, dim, keepdim, dtype, True)


@impl(aten.sum.default)
def _sum_all(func, self, dtype=None):
    out = torch.empty((), dtype=dtype or self.dtype, device=self.device)
    acc = torch.empty((), dtype=torch.float32, device=self.device)
    fill_(acc, 0.0)
    reduce_sum(self, list(range(self.dim())), acc.view(1))
    return ew(out, [acc], EW_COPY)


# ---- BatchNorm -------------------------------------------------------------------
def _rows_ld(t: torch.Tensor) -> Optional[int]:
    """Row stride (elements) when t is an [M, C] row matrix in memory -- channels-last 4-D or 2-D with unit-stride
    channels, compact or a channel slice of a wider one (a concat buffer's tail, a padded conv output's first C
    channels) -- with 16-B channel vectors (8-B for bf16 C % 8 != 0); else None."""
    if t.dim() == 4:
        ld = _row_stride(t.permute(0, 2, 3, 1))
    elif t.dim() == 2 and t.stride(1) == 1:
        ld = t.stride(0) if t.shape[0] > 1 else t.shape[1]
    else:
        return None
    C = t.shape[1]
    if ld is None or C % 4 or ld < C or t.dtype not in (torch.float32, torch.bfloat16) or t.numel() == 0:
        return None
    align = 16 if (t.dtype == torch.float32 or C % 8 == 0) else 8
    if t.data_ptr() % align or (ld * t.element_size()) % align:
        return None
    return int(ld)


def _cl_rows(t: torch.Tensor) -> bool:
    return _rows_ld(t) is not None


def _same_geom(a: torch.Tensor, b: torch.Tensor) -> bool:
    return a.shape == b.shape and a.stride() == b.stride()


def _same(a, b) -> bool:
    return isinstance(a, torch.Tensor) and a.data_ptr() == b.data_ptr() and _same_geom(a, b) and a.dtype == b.dtype


class _PendingBN:
    """A BatchNorm output whose apply pass (x * scale + shift [+ res]) has not run yet: if the next op is
    a residual add of it (identity or projection shortcut), the add joins the pending pass; if the next
    op is its ReLU, everything becomes one pass (EW_FMA_RELU / EW_FMA_ADD_RELU); any other op
    materialises it first."""
    __slots__ = ("out", "x", "scale", "shift", "res")

    def __init__(self, out, x, scale, shift, res=None):
        self.out, self.x, self.scale, self.shift, self.res = out, x, scale, shift, res

    def inputs(self):
        return [self.x, self.scale, self.shift] + ([] if self.res is None else [self.res])

    def rounding(self) -> float:
        # the unfused BN stores its output before the add reads it: round there too (bit-identical results)
        return 1.0 if self.res is not None and self.out.dtype == torch.bfloat16 else 0.0

    def materialize(self):
        ew(self.out, self.inputs(), EW_FMA if self.res is None else EW_FMA_ADD, 0.0, self.rounding())

    def relu(self, out):
        return ew(out, self.inputs(), EW_FMA_RELU if self.res is None else EW_FMA_ADD_RELU, 0.0, self.rounding())


def _bn_add_partner(pend, args, kwargs=None):
    """The other operand of ``add.Tensor(a, b)`` when one operand is the pending BN output and the pair can
    join the pending pass (no alpha, same geometry and dtype, no residual taken yet); else None."""
    if pend is None or pend.res is not None or len(args) < 2 or len(args) > 2 or (kwargs and kwargs.get("alpha", 1) != 1):
        return None
    a, b = args[0], args[1]
    if not (isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor)):
        return None
    o = b if _same(a, pend.out) else a if _same(b, pend.out) else None
    if o is None or o is pend.out or o.dtype != pend.out.dtype or not _same_geom(o, pend.out):
        return None
    return o


def _mode_pending_bn(t):
    mode = NativeMode.current
    if mode is None or mode._pend_bn is None or not _same(t, mode._pend_bn.out):
        return None
    pend, mode._pend_bn = mode._pend_bn, None
    return pend


@impl(aten.native_batch_norm.default)
def _bn(func, input, weight, bias, running_mean, running_var, training, momentum, eps):
    x = input
    C = x.shape[1]
    dev = x.device
    M = x.numel() // C
    f32 = dict(dtype=torch.float32, device=dev)
    scale, shift_out = torch.empty(C, **f32), torch.empty(C, **f32)
    nat = _nat()
    mode = NativeMode.current
    ldx = _rows_ld(x)
    rows = ldx is not None
    if mode is not None and not (training and rows):
        mode._flush_ctr()
    if training and rows:
        # channels-last rows: moments (slab partials) + ONE finalize that also derives the coefficients and
        # the running stats (2 launches; the generic path below takes 4)
        save_mean, save_invstd = torch.empty(C, **f32), torch.empty(C, **f32)
        p = lambda t: 0 if t is None else t.data_ptr()   # noqa: E731
        part = torch.empty(int(nat.z_reduce_rows_ws_floats(M, C)), **f32)
        ctr = mode._take_ctr() if mode is not None else None
        nat.z_bn_rows_fwd(_st(dev), x.data_ptr(), _DT[x.dtype], ldx, p(running_mean), C, M, part.data_ptr(), part.numel(),
                          p(weight), p(bias), p(running_mean), p(running_var), float(eps),
                          float(momentum if momentum is not None else 0.1), save_mean.data_ptr(), save_invstd.data_ptr(),
                          scale.data_ptr(), shift_out.data_ptr(), p(ctr))
    elif training:
        acc = torch.empty(2 * C, **f32)
        fill_(acc, 0.0)
        dims = [0] + list(range(2, x.dim()))
        # moments of (x - running_mean): no catastrophic cancellation in E[d^2] - E[d]^2
        reduce_sum(x, dims, acc[:C], RD_SUMSQ_SHIFT, shift=running_mean, acc2=acc[C:])
        save_mean, save_invstd = torch.empty(C, **f32), torch.empty(C, **f32)
        p = lambda t: 0 if t is None else t.data_ptr()   # noqa: E731
        nat.z_bn_fwd_coeffs(_st(dev), acc.data_ptr(), acc[C:].data_ptr(), p(running_mean), C, M, p(weight), p(bias),
                            p(running_mean), p(running_var), float(eps), float(momentum if momentum is not None else 0.1),
                            1, save_mean.data_ptr(), save_invstd.data_ptr(), scale.data_ptr(), shift_out.data_ptr())
    else:
        p = lambda t: 0 if t is None else t.data_ptr()   # noqa: E731
        nat.z_bn_fwd_coeffs(_st(dev), 0, 0, 0, C, M, p(weight), p(bias), p(running_mean), p(running_var), float(eps),
                            0.0, 0, 0, 0, scale.data_ptr(), shift_out.data_ptr())
        save_mean = torch.empty(0, **f32)
        save_invstd = torch.empty(0, **f32)
    bshape = [1, C] + [1] * (x.dim() - 2)
    out = torch.empty_like(x)      # channels-last compact even for a row-strided x (empty_like of a non-dense view)
    if mode is not None and mode.fuse and rows and _cl_rows(out):
        mode._pend_bn = _PendingBN(out, x, scale.view(bshape), shift_out.view(bshape))
    else:
        ew(out, [x, scale.view(bshape), shift_out.view(bshape)], EW_FMA)
    return out, save_mean, save_invstd


@impl(aten.miopen_batch_norm.default)
def _bn_miopen(func, input, weight, bias, running_mean, running_var, training, exponential_average_factor, epsilon):
    # ATen's batch_norm picks the MIOpen variant for CUDA inputs before dispatch; same op, same saved
    # tensors (mean, invstd) as the native_batch_norm path -- only our backward reads them
    return _bn(None, input, weight, bias, running_mean, running_var, training, exponential_average_factor, epsilon)


@impl(aten.miopen_batch_norm_backward.default)
def _bn_miopen_bwd(func, input, grad_output, weight, running_mean, running_var, save_mean, save_var, epsilon):
    return _bn_bwd(None, grad_output, input, weight, running_mean, running_var, save_mean, save_var, True, epsilon,
                   [True, weight is not None, weight is not None])


@impl(aten.native_batch_norm_backward.default)
def _bn_bwd(func, grad_out, input, weight, running_mean, running_var, save_mean, save_invstd, train, eps,
            output_mask):
    if not train:
        return None
    x, g = input, grad_out
    C = x.shape[1]
    dev = x.device
    M = x.numel() // C
    f32 = dict(dtype=torch.float32, device=dev)
    k, bb, cc = torch.empty(C, **f32), torch.empty(C, **f32), torch.empty(C, **f32)
    gw = (_param_grad(weight) if output_mask[1] else None) if weight is not None else None
    gw = gw if gw is not None else (torch.empty(C, **f32) if output_mask[1] else None)
    gb = (_param_grad(weight, bias=True) if output_mask[2] else None) if weight is not None else None
    gb = gb if gb is not None and gb.shape[0] == C else (torch.empty(C, **f32) if output_mask[2] else None)
    p = lambda t: 0 if t is None else t.data_ptr()   # noqa: E731
    mode = NativeMode.current
    thr = None
    if mode is not None and mode._pend_thr is not None and _same(g, mode._pend_thr.out):
        thr, mode._pend_thr = mode._pend_thr, None   # this BN's ReLU backward, fused into its sums and apply
        mode._defer(thr.out, thr.materialize)
        mode.fused["relu_bwd+bn_bwd"] += 1
        g = thr.grad
    ldg, ldx = _rows_ld(g), _rows_ld(x)
    ldf = _rows_ld(thr.relu_out) if thr else 0
    if ldg is not None and ldx is not None and ldf is not None and g.shape == x.shape:
        nat = _nat()
        part = torch.empty(int(nat.z_reduce_rows_ws_floats(M, C)), **f32)
        nat.z_bn_rows_bwd(_st(dev), g.data_ptr(), _DT[g.dtype], ldg, x.data_ptr(), _DT[x.dtype], ldx,
                          thr.relu_out.data_ptr() if thr else 0, _DT[thr.relu_out.dtype] if thr else 0, ldf,
                          thr.thr if thr else 0.0, save_mean.data_ptr(), save_invstd.data_ptr(), p(weight), C, M,
                          part.data_ptr(), part.numel(), k.data_ptr(), bb.data_ptr(), cc.data_ptr(), p(gw), p(gb))
    else:
        if thr is not None:
            thr.materialize()
            g, thr = thr.out, None
        acc = torch.empty(2 * C, **f32)
        fill_(acc, 0.0)
        dims = [0] + list(range(2, x.dim()))
        reduce_sum(g, dims, acc[:C], RD_DOT_SHIFT, b=x, shift=save_mean, acc2=acc[C:])
        _nat().z_bn_bwd_coeffs(_st(dev), acc.data_ptr(), acc[C:].data_ptr(), save_mean.data_ptr(),
                               save_invstd.data_ptr(), p(weight), C, M, k.data_ptr(), bb.data_ptr(), cc.data_ptr(),
                               p(gw), p(gb))
    gi = None
    if output_mask[0]:
        bshape = [1, C] + [1] * (x.dim() - 2)
        gi = torch.empty_like(x)
        ins = [g, k.view(bshape), x, bb.view(bshape), cc.view(bshape)] + ([thr.relu_out] if thr is not None else [])
        pend = _PendingBNB(gi, ins, thr.thr if thr is not None else 0.0)
        if mode is not None and mode.fuse:
            mode._pend_bnb = pend            # autograd's accumulation add of this gradient may join the pass
        else:
            pend.materialize()
    if gw is not None and weight is not None and gw.dtype != weight.dtype:
        gw = ew(torch.empty_like(weight), [gw], EW_COPY)
    return gi, gw, gb


# ---- pooling ---------------------------------------------------------------------
def _pair(v, default=None):
    if v is None or (isinstance(v, (list, tuple)) and len(v) == 0):
        return default
    if isinstance(v, int):
        return (v, v)
    return (int(v[0]), int(v[1] if len(v) > 1 else v[0]))


@impl(aten.avg_pool2d.default)
def _avgpool(func, self, kernel_size, stride=(), padding=0, ceil_mode=False, count_include_pad=True,
             divisor_override=None):
    k = _pair(kernel_size)
    s = _pair(stride, k)
    p = _pair(padding)
    out = _alloc_like_meta(func, (self, kernel_size, stride, padding, ceil_mode, count_include_pad, divisor_override),
                           {}, self.device)
    _nat().z_pool_fwd(_st(self.device), zd(self), zd(out), None, k[0], k[1], s[0], s[1], p[0], p[1],
                      int(count_include_pad), int(divisor_override or 0), 0)
    return out


@impl(aten.avg_pool2d_backward.default)
def _avgpool_bwd(func, grad_output, self, kernel_size, stride, padding, ceil_mode, count_include_pad,
                 divisor_override):
    k = _pair(kernel_size)
    s = _pair(stride, k)
    p = _pair(padding)
    gi = torch.empty_like(self)
    _nat().z_pool_bwd(_st(self.device), zd(gi), zd(grad_output), None, k[0], k[1], s[0], s[1], p[0], p[1],
                      int(count_include_pad), int(divisor_override or 0), 0)
    return gi


@impl(aten.max_pool2d_with_indices.default)
def _maxpool(func, self, kernel_size, stride=(), padding=0, dilation=1, ceil_mode=False):
    if _pair(dilation) != (1, 1):
        return None
    k = _pair(kernel_size)
    s = _pair(stride, k)
    p = _pair(padding)
    out, idx = _alloc_like_meta(func, (self, kernel_size, stride, padding, dilation, ceil_mode), {}, self.device)
    _nat().z_pool_fwd(_st(self.device), zd(self), zd(out), zd(idx), k[0], k[1], s[0], s[1], p[0], p[1], 0, 0, 1)
    return out, idx


@impl(aten.max_pool2d_with_indices_backward.default)
def _maxpool_bwd(func, grad_output, self, kernel_size, stride, padding, dilation, ceil_mode, indices):
    k = _pair(kernel_size)
    s = _pair(stride, k)
    p = _pair(padding)
    gi = torch.empty_like(self)
    _nat().z_pool_bwd(_st(self.device), zd(gi), zd(grad_output), zd(indices), k[0], k[1], s[0], s[1], p[0], p[1], 0, 0,
                      1)
    return gi


# ---- GEMM ---------------------------------------------------------------------------
def _gemm_out_dtype(*ts):
    return torch.float32 if any(t is not None and t.dtype == torch.float32 for t in ts) else ts[0].dtype


@impl(aten.mm.default)
def _mm(func, self, mat2):
    out = torch.empty(self.shape[0], mat2.shape[1], dtype=_gemm_out_dtype(self, mat2), device=self.device)
    _nat().z_gemm(_st(self.device), zd(self), zd(mat2), zd(out), None, 1.0, 0.0)
    return out


@impl(aten.addmm.default)
def _addmm(func, bias, mat1, mat2, beta=1, alpha=1):
    out = torch.empty(mat1.shape[0], mat2.shape[1], dtype=_gemm_out_dtype(mat1, mat2, bias), device=mat1.device)
    _nat().z_gemm(_st(mat1.device), zd(mat1), zd(mat2), zd(out), zd(bias), float(alpha), float(beta))
    return out


# ---- log-softmax / NLL --------------------------------------------------------------
@impl(aten._log_softmax.default)
def _log_softmax(func, self, dim, half_to_float):
    if self.dim() != 2 or dim % 2 != 1:
        return None
    out = _alloc_like_meta(func, (self, dim, half_to_float), {}, self.device)
    _nat().z_log_softmax(_st(self.device), zd(self), zd(out), 0, None)
    return out


@impl(aten._log_softmax_backward_data.default)
def _log_softmax_bwd(func, grad_output, output, dim, input_dtype):
    if output.dim() != 2 or dim % 2 != 1:
        return None
    out = torch.empty(output.shape, dtype=input_dtype, device=output.device)
    _nat().z_log_softmax(_st(output.device), zd(output), zd(out), 1, zd(grad_output))
    return out


@impl(aten.nll_loss_forward.default)
def _nll_fwd(func, self, target, weight, reduction, ignore_index):
    if weight is not None or self.dim() != 2 or reduction not in (1, 2):
        return None
    out = torch.empty((), dtype=self.dtype, device=self.device)
    tw = torch.empty((), dtype=self.dtype, device=self.device)
    _nat().z_nll_fwd(_st(self.device), zd(self), target.data_ptr(), target.stride(0), int(ignore_index),
                     int(reduction == 1), out.data_ptr(), int(out.dtype == torch.bfloat16), tw.data_ptr(),
                     int(tw.dtype == torch.bfloat16))
    return out, tw


@impl(aten.nll_loss_backward.default)
def _nll_bwd(func, grad_output, self, target, weight, reduction, ignore_index, total_weight):
    if weight is not None or self.dim() != 2 or reduction not in (1, 2):
        return None
    gx = torch.empty_like(self)
    _nat().z_nll_bwd(_st(self.device), zd(gx), grad_output.data_ptr(), int(grad_output.dtype == torch.bfloat16),
                     total_weight.data_ptr(), int(total_weight.dtype == torch.bfloat16), target.data_ptr(),
                     target.stride(0), int(ignore_index), int(reduction == 1))
    return gx


# ---- RNG (dropout / drop-connect) -----------------------------------------------------
@impl(aten.bernoulli_.float)
def _bernoulli_(func, self, p=0.5, generator=None):
    mode = NativeMode.current
    ew(self, [], EW_BERN, float(p), seed=mode.seed, ctr=mode.rng_ctr(self.device))
    _nat().z_ctr_bump(_st(self.device), mode.rng_ctr(self.device).data_ptr())
    return self


@impl(aten.native_dropout.default)
def _native_dropout(func, input, p, train):
    mask = torch.empty_like(input)
    if not train or p == 0:
        fill_(mask, 1.0)
        return ew(torch.empty_like(input), [input], EW_COPY), mask
    # the mask is kept in the input's dtype (0 / 1): only native_dropout_backward below reads it
    _bernoulli_(None, mask, 1.0 - float(p))
    out = ew(torch.empty_like(input), [input, mask], EW_MUL)
    return ew(out, [out], EW_MULS, 1.0 / (1.0 - float(p))), mask


@impl(aten.native_dropout_backward.default)
def _native_dropout_bwd(func, grad_output, mask, scale):
    out = ew(torch.empty_like(grad_output), [grad_output, mask], EW_MUL)
    return ew(out, [out], EW_MULS, float(scale))


# ---- convolution ----------------------------------------------------------------------
def _cl_bf16(x: torch.Tensor, rows: bool = False) -> torch.Tensor:
    """channels-last contiguous bf16 (NCHW-shaped) -- a no-op for the engine's activations.  ``rows``: a
    row-strided channels-last view (a channel slice) passes as is too (the MFMA conv paths pad / copy it
    through :func:`_pad_c`, which reads row strides)."""
    if x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last):
        return x
    if rows and x.dtype == torch.bfloat16 and x.dim() == 4 and _row_stride(_nhwc(x)) is not None:
        return x
    out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    return ew(out, [x], EW_COPY)


def _conv_kind(C, O, groups, k, stride, pad, dil):
    square = k[0] == k[1] and stride[0] == stride[1] and pad[0] == pad[1]
    if dil != (1, 1) or not square or stride[0] not in (1, 2) or k[0] > 7:
        return "gconv"
    if groups == C == O and C % 8 == 0 and C <= 2048 and k[0] in (3, 5, 7) and C * k[0] * k[0] * 4 <= 128 * 1024:
        return "dw"
    if groups == C == O and C % 4 == 0 and C <= 2040 and k[0] in (3, 5, 7) and CV.pad8(C) * k[0] * k[0] * 4 <= 128 * 1024:
        # depthwise on an off-grid width (PNASNetA's 44 / 88 / 176 channels): the depthwise kernels on channels
        # zero-padded to 8 (input, weights, output gradient), results read back as row-strided views
        return "dwpad"
    if groups <= 8:
        # one MFMA implicit GEMM per group; channel counts off the 8-grid (stems, DenseNet growth widths,
        # ShuffleNet g2/g3 widths) are zero-padded
        return "mfma"
    if C % 8 == 0 and O % 8 == 0 and C // groups <= 32 and C <= 1024 and O <= 1024:
        # many narrow groups (DPN cardinality 32, ResNeXt 32x4d, RegNet group width 8): one dense MFMA conv over a
        # block-diagonal weight image does groups-times the FLOPs but runs on the matrix cores -- the direct VALU
        # kernel (gconv) spent 8.9 of DPN26's 17 ms per step on its 3- / 6- / 12-channel groups
        return "gdense"
    return "gconv"


def _row_stride(t: torch.Tensor) -> Optional[int]:
    """Row stride (elements) when ``t`` [..., C] is evenly spaced rows of unit-stride channels (a compact tensor
    or a channel slice of one), else None."""
    if t.dim() < 2 or t.stride(-1) != 1:
        return None
    ld = expect = None
    for d in range(t.dim() - 2, -1, -1):
        if t.shape[d] == 1:
            continue
        if ld is None:
            ld, expect = t.stride(d), t.stride(d) * t.shape[d]
        elif t.stride(d) != expect:
            return None
        else:
            expect *= t.shape[d]
    return int(ld) if ld is not None else int(t.shape[-1])


def _pad_c(t: torch.Tensor, c8: int, cache: bool = False) -> torch.Tensor:
    """NHWC bf16 [.., C] (possibly a channel slice) -> contiguous [.., c8], zero channels C..c8.  ``cache``:
    reuse / keep the padded copy for the rest of the NativeMode block (a conv's input is padded by its
    forward and again by its weight gradient)."""
    C = t.shape[-1]
    if C == c8 and t.is_contiguous():
        return t
    mode = NativeMode.current
    key = ("pad", t.data_ptr(), tuple(t.shape), tuple(t.stride()), c8)
    if cache and mode is not None and key in mode._wcache:
        return mode._wcache[key][1]
    out = torch.empty(*t.shape[:-1], c8, dtype=torch.bfloat16, device=t.device)
    rows = t.numel() // C if C else 0
    if t.dtype == torch.bfloat16 and rows and _row_stride(t) is not None:
        _nat().z_pad_rows(_st(t.device), t.data_ptr(), _row_stride(t), C, out.data_ptr(), c8, rows)   # one launch
    else:
        if c8 > C:
            fill_(out[..., C:], 0.0)
        ew(out[..., :C], [t], EW_COPY)
    if cache and mode is not None:
        mode._wcache[key] = (t, out)
    return out


def _unpad_c(t: torch.Tensor, c: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The first ``c`` channels of a channel-padded NHWC result: copied into ``out`` when given, else the
    row-strided view itself -- its consumers (BN row passes, elementwise / concat copies, the next conv's
    channel pad) all read row strides, so the compacting copy is not needed."""
    if out is None:
        return t if t.shape[-1] == c else t[..., :c]
    return ew(out, [t[..., :c]], EW_COPY)


def _pad_o(w32: torch.Tensor, o8: int) -> torch.Tensor:
    """fp32 [O, C, R, S] -> contiguous [o8, C, R, S] with zero filters O..o8."""
    O = w32.shape[0]
    if O == o8 and w32.is_contiguous():
        return w32
    out = torch.empty(o8, *w32.shape[1:], dtype=torch.float32, device=w32.device)
    if o8 > O:
        fill_(out[O:], 0.0)
    ew(out[:O], [w32], EW_COPY)
    return out


def _packed(w32, O8: int, C8: int, st: int, pd: int, need_wd: bool = False, groups: int = 1):
    """bf16 [O8, R, S, C8] conv image of fp32 ``w32`` (and with ``need_wd`` its DGRAD image), packed once per
    NativeMode block: the forward packs, the backward of the same step reuses (the weights only change at
    the SGD, outside the block).  Weights living in the trainer's flat parameter storage
    (:attr:`NativeMode.stable_storage`) are remembered: the next block packs all of them in one multi-tensor
    launch at its first conv (and all DGRAD images at its first conv backward) instead of one launch each."""
    mode = NativeMode.current
    cache = mode._wcache if mode is not None else None
    key = (w32.data_ptr(), tuple(w32.shape), tuple(w32.stride()), O8, C8, st, pd, groups)
    if mode is not None:
        if not mode._prepacked:
            mode._prepacked = True
            mode._prepack(wd=False)
        if need_wd and not mode._prepacked_wd:
            mode._prepacked_wd = True
            mode._prepack(wd=True)
        if mode.stable_storage and w32.untyped_storage().data_ptr() == mode.stable_storage:
            mode._pack_plan.setdefault(key, w32)
            if need_wd:
                mode._wd_plan.setdefault(key, w32)
    ent = cache.get(key) if cache is not None else None
    if ent is None:
        ent = {}
        if cache is not None:
            cache[key] = (w32, ent)          # holds w32: the pointer key stays valid for the block
    else:
        ent = ent[1]
    if "wp" not in ent:   # zero filters O..O8 (and a grouped conv's off-diagonal blocks): same launch
        ent["wp"] = CV.pack_weight(w32.contiguous(), c_pad=C8, o_pad=O8, groups=groups)
    if need_wd and "wd" not in ent:
        ent["wd"] = _wd_image(w32, O8, C8, st, pd)
        CV.dgrad_pack_weights([(_pad_o(w32, O8), ent["wd"], st, pd, C8)])
    return ent["wp"], ent.get("wd")


def _wd_image(w32, O8, C8, st, pd):
    return torch.empty(CV.dgrad_image_numel((O8,) + tuple(w32.shape[1:]), C8), dtype=torch.bfloat16,
                       device=w32.device)


def _dense_fwd(xh, w32, st, pd, out=None, groups: int = 1):
    """One group: y [N,P,Q,Og] = conv(xh [N,H,W,Cg] NHWC bf16 (a view is fine), w32 [Og,Cg,R,S]).  ``groups`` > 1:
    the whole grouped conv as one dense MFMA conv over a block-diagonal weight image (xh holds all channels)."""
    Og, Cg, R, S = w32.shape
    C8, O8 = CV.pad8(Cg * groups), CV.pad8(Og)
    xp = _pad_c(xh, C8, cache=True)
    wp, _ = _packed(w32, O8, C8, st, pd, groups=groups)
    y = CV.conv2d_fwd(xp, wp, st, pd, ws=_ws(xh.device, CV.fd_ws_floats(xp.shape, O8, R, S, st, pd)))
    return _unpad_c(y, Og, out)


def _dense_bwd(xh, gy, w32, st, pd, need_dx, need_dw, dx_out=None, dw_out=None, groups: int = 1):
    """One group's data / weight gradients; dx written into ``dx_out`` (NHWC view) when given.  ``groups`` > 1:
    the densified grouped conv of :func:`_dense_fwd` (the DGRAD reads the block-diagonal image; the WGRAD
    reduction keeps each filter's own group of the dense gradient)."""
    Og, Cg, R, S = w32.shape
    N, H, W = xh.shape[:3]
    C8, O8 = CV.pad8(Cg * groups), CV.pad8(Og)
    gyp = _pad_c(gy, O8)
    dx = dw = None
    if need_dx:
        # (O % 64 only: the stride-1 GEN DGRAD of the CNN engine measured 14 % slower on densenet_cifar here, where
        # no BN sums ride in its epilogue -- profiles/r6_zoo/routing_ab/)
        wp, wd = _packed(w32, O8, C8, st, pd, need_wd=groups == 1 and CV.dgrad_eligible(O8), groups=groups)
        xs = (N, H, W, C8)
        d = CV.conv2d_dgrad(gyp, wp, xs, st, pd, wd=wd, ws=_ws(xh.device, CV.fd_ws_floats(xs, O8, R, S, st, pd)))
        dx = _unpad_c(d, Cg * groups, dx_out)
    if need_dw:   # the padded filters O..O8 never leave the reduction (Ow): no slice copy
        out = dw_out if dw_out is not None and dw_out.is_contiguous() else None
        xp = _pad_c(xh, C8, cache=True)
        part, wred = _wred_part(out, CV.wgrad_ws_floats(xp.shape, O8, R, S, st, pd, Cg))
        # (no library-GEMM route here: 1-2.5 % slower on RegNetX / SimpleDLA / DenseNet121, profiles/r6_zoo/routing_ab/)
        dw = CV.conv2d_wgrad(xp, gyp, R, S, st, pd, Cw=Cg, Ow=Og, groups=groups, out=out, ws=part, deferred=wred,
                             lib_gemm=False)
        if dw_out is not None and dw.data_ptr() != dw_out.data_ptr():
            dw = ew(dw_out, [dw], EW_COPY)
    return dx, dw


def _wred_part(out: Optional[torch.Tensor], floats: int):
    """(workspace, deferred list) for a WGRAD into ``out``: while a mode runs, a WGRAD that writes a trainer's flat
    gradient slot keeps its split-K partials in a buffer of its own and appends its reduction to the mode's list --
    ONE wgrad_reduce_multi launch (per 32) sums them all when anything reads a pending slot, or at the mode's flush
    (bit-identical to the per-conv reduce: conv_igemm.hip wgrad_reduce.h; ~120 launches per DenseNet step).
    (None, None): reduce right away in the shared workspace."""
    mode = NativeMode.current
    if mode is None or not mode.defer_wred or out is None or floats <= 0:
        return None, None
    part = torch.empty(floats, dtype=torch.float32, device=out.device)
    mode._wred_keep.append(part)
    mode._wred_ptrs.add(out.data_ptr())
    return part, mode._wred


def _dw_padded_weight(w32: torch.Tensor, C8: int) -> torch.Tensor:
    """fp32 [C8, 1, R, R] depthwise weights with zero channels C..C8, made once per NativeMode block."""
    mode = NativeMode.current
    key = ("dwpad", w32.data_ptr(), tuple(w32.shape), C8)
    if mode is not None and key in mode._wcache:
        return mode._wcache[key][1]
    wp = _pad_o(w32.contiguous(), C8)
    if mode is not None:
        mode._wcache[key] = (w32, wp)
    return wp


def _nchw(t_nhwc: torch.Tensor) -> torch.Tensor:
    return t_nhwc.permute(0, 3, 1, 2)


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 2, 3, 1)


def _ws(dev, floats):
    return CV.wgrad_workspace(dev, floats) if floats > 0 else None


def _param_grad(w: Optional[torch.Tensor], bias: bool = False) -> Optional[torch.Tensor]:
    """The trainer's flat-gradient slot of parameter ``w`` (``bias``: of the bias that belongs to weight ``w``), a
    view of :attr:`NativeMode.grad_flat` shaped like the parameter, handed out once per block.  A native backward
    writes the parameter gradient straight into it and autograd's AccumulateGrad adopts the tensor as ``p.grad``
    (the trainer clears ``p.grad`` before backward, :meth:`fedmi.engine.torch_engine.TorchTrainer._step_body`):
    no accumulation pass per parameter (~360 launches per DenseNet step).  None: allocate as usual."""
    mode = NativeMode.current
    if (mode is None or mode.grad_flat is None or not isinstance(w, torch.Tensor) or not w.is_cuda
            or w.dtype != torch.float32 or not w.is_contiguous() or w.untyped_storage().data_ptr() != mode.stable_storage):
        return None
    off, n, shape = w.storage_offset(), w.numel(), w.shape
    if bias:
        ent = mode.bias_of.get(off)
        if ent is None:
            return None
        off, n = ent
        shape = (n,)
    if off + n > mode.grad_flat.numel() or off in mode._grad_taken:
        return None
    mode._grad_taken.add(off)
    return mode.grad_flat[off:off + n].view(shape)


@impl(aten.convolution.default)
def _conv(func, input, weight, bias, stride, padding, dilation, transposed, output_padding, groups):
    if transposed or input.dim() != 4:
        return None
    k = tuple(weight.shape[2:])
    st, pd, dl = _pair(stride), _pair(padding), _pair(dilation)
    N, C, H, W = input.shape
    O = weight.shape[0]
    kind = _conv_kind(C, O, groups, k, st, pd, dl)
    dev = input.device
    w32 = weight if weight.dtype == torch.float32 else ew(torch.empty(weight.shape, device=dev), [weight], EW_COPY)
    if kind in ("mfma", "dw", "gdense", "dwpad"):
        xh = _nhwc(_cl_bf16(input, rows=kind != "dw"))
        if kind == "dwpad":
            C8 = CV.pad8(C)
            y = CV.dwconv_fwd(_pad_c(xh, C8, cache=True), _dw_padded_weight(w32, C8), st[0], pd[0])[..., :C]
        elif kind == "dw":
            y = CV.dwconv_fwd(xh, w32.contiguous(), st[0], pd[0])
        elif kind == "gdense":
            y = _dense_fwd(xh, w32, st[0], pd[0], groups=groups)
        elif groups == 1:
            y = _dense_fwd(xh, w32, st[0], pd[0])
        else:
            P = (H + 2 * pd[0] - k[0]) // st[0] + 1
            Q = (W + 2 * pd[1] - k[1]) // st[1] + 1
            y = torch.empty(N, P, Q, O, dtype=torch.bfloat16, device=dev)
            Cg, Og = C // groups, O // groups
            for g in range(groups):
                _dense_fwd(xh[..., g * Cg:(g + 1) * Cg], w32[g * Og:(g + 1) * Og], st[0], pd[0],
                           out=y[..., g * Og:(g + 1) * Og])
        out = _nchw(y)
    else:
        P = (H + 2 * pd[0] - dl[0] * (k[0] - 1) - 1) // st[0] + 1
        Q = (W + 2 * pd[1] - dl[1] * (k[1] - 1) - 1) // st[1] + 1
        if dl != (1, 1):
            return None
        out = torch.empty(N, O, P, Q, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        _nat().z_gconv(_st(dev), 0, zd(input), zd(w32), zd(out), int(groups), st[0], st[1], pd[0], pd[1])
    if bias is not None:
        ew(out, [out, bias.view(1, O, 1, 1)], EW_ADD, 1.0)
    return out


@impl(aten.convolution_backward.default)
def _conv_bwd(func, grad_output, input, weight, bias_sizes, stride, padding, dilation, transposed, output_padding,
              groups, output_mask):
    if transposed or input.dim() != 4:
        return None
    k = tuple(weight.shape[2:])
    st, pd, dl = _pair(stride), _pair(padding), _pair(dilation)
    N, C, H, W = input.shape
    O = weight.shape[0]
    kind = _conv_kind(C, O, groups, k, st, pd, dl)
    dev = input.device
    w32 = weight if weight.dtype == torch.float32 else ew(torch.empty(weight.shape, device=dev), [weight], EW_COPY)
    gi = gw = gb = None
    gw_slot = _param_grad(weight) if output_mask[1] else None
    if kind in ("mfma", "dw", "gdense", "dwpad"):
        xh = _nhwc(_cl_bf16(input, rows=kind != "dw"))
        gy = _nhwc(_cl_bf16(grad_output, rows=kind != "dw"))
        if kind == "dwpad":
            C8 = CV.pad8(C)
            gyp = _pad_c(gy, C8)
            if output_mask[0]:
                gi = _nchw(CV.dwconv_dgrad(gyp, _dw_padded_weight(w32, C8), (N, H, W, C8), st[0], pd[0])[..., :C])
            if output_mask[1]:
                gw8 = CV.dwconv_wgrad(_pad_c(xh, C8, cache=True), gyp, k[0], st[0], pd[0])
                gw = ew(gw_slot, [gw8[:C]], EW_COPY) if gw_slot is not None else gw8[:C]
        elif kind == "gdense":
            dx, gw = _dense_bwd(xh, gy, w32, st[0], pd[0], output_mask[0], output_mask[1], dw_out=gw_slot,
                                groups=groups)
            gi = _nchw(dx) if dx is not None else None
        elif kind == "dw":
            if output_mask[0]:
                gi = _nchw(CV.dwconv_dgrad(gy, w32.contiguous(), xh.shape, st[0], pd[0]))
            if output_mask[1]:
                part, wred = _wred_part(gw_slot, CV.dwconv_ws_floats(xh.shape, k[0], st[0], pd[0]))
                gw = CV.dwconv_wgrad(xh, gy, k[0], st[0], pd[0], out=gw_slot, ws=part, deferred=wred)
        elif groups == 1:
            dx, gw = _dense_bwd(xh, gy, w32, st[0], pd[0], output_mask[0], output_mask[1], dw_out=gw_slot)
            gi = _nchw(dx) if dx is not None else None
        else:
            Cg, Og = C // groups, O // groups
            gih = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=dev) if output_mask[0] else None
            gw = (gw_slot if gw_slot is not None else torch.empty(O, Cg, k[0], k[1], dtype=torch.float32, device=dev)) \
                if output_mask[1] else None
            for g in range(groups):
                _dense_bwd(xh[..., g * Cg:(g + 1) * Cg], gy[..., g * Og:(g + 1) * Og], w32[g * Og:(g + 1) * Og],
                           st[0], pd[0], output_mask[0], output_mask[1],
                           dx_out=gih[..., g * Cg:(g + 1) * Cg] if gih is not None else None,
                           dw_out=gw[g * Og:(g + 1) * Og] if gw is not None else None)
            gi = _nchw(gih) if gih is not None else None
        if gi is not None and input.dtype != torch.bfloat16:
            gi = ew(torch.empty_like(input), [gi], EW_COPY)
    else:
        if dl != (1, 1):
            return None
        if output_mask[0]:
            gi = torch.empty_like(input)
            _nat().z_gconv(_st(dev), 1, zd(gi), zd(w32), zd(grad_output), int(groups), st[0], st[1], pd[0], pd[1])
        if output_mask[1]:
            gw = gw_slot if gw_slot is not None else torch.empty(w32.shape, dtype=torch.float32, device=dev)
            P, Q = grad_output.shape[2], grad_output.shape[3]
            wsf = int(_nat().z_gconv_wgrad_ws_floats(N, P, Q, gw.numel()))
            ws = CV.wgrad_workspace(dev, wsf)
            _nat().z_gconv(_st(dev), 2, zd(input), zd(gw), zd(grad_output), int(groups), st[0], st[1], pd[0], pd[1],
                           ws.data_ptr(), ws.numel())
    if gw is not None and gw.dtype != weight.dtype:
        gw = ew(torch.empty_like(weight), [gw], EW_COPY)
    if output_mask[2]:
        gb = _param_grad(weight, bias=True)
        if gb is None or gb.shape[0] != O:
            gb = torch.empty(O, dtype=weight.dtype, device=dev)
        if _rowmajor_out(gb):
            reduce_sum(grad_output, [0, 2, 3], None, out=gb)
        else:
            acc = torch.empty(O, dtype=torch.float32, device=dev)
            fill_(acc, 0.0)
            reduce_sum(grad_output, [0, 2, 3], acc)
            ew(gb, [acc], EW_COPY)
    return gi, gw, gb


# ---------------------------------------------------------------------------- the mode
def _ops(*names):
    out = set()
    for n in names:
        pkt, _, ov = n.partition(".")
        op = getattr(getattr(aten, pkt, None), ov or "default", None)
        if op is not None:
            out.add(op)
    return out


_PASSTHROUGH = _ops(
    "view", "_unsafe_view", "expand", "t", "transpose.int", "permute", "slice.Tensor", "select.int", "detach",
    "alias", "unsqueeze", "squeeze.dim", "squeeze", "squeeze.dims", "as_strided", "split.Tensor",
    "split_with_sizes", "chunk", "unbind.int", "empty.memory_format", "empty_like", "empty_strided", "new_empty",
    "new_empty_strided", "reshape", "flatten.using_ints", "_reshape_alias", "lift_fresh", "narrow", "unflatten.int",
    "_local_scalar_dense", "is_same_size", "as_strided_", "view.dtype", "set_.source_Storage_storage_offset",
)


_BN_FWD = _ops("native_batch_norm", "miopen_batch_norm")
# in-place ops among the native impls (their first argument is written)
_INPLACE = _ops("add_.Tensor", "sub_.Tensor", "mul_.Tensor", "div_.Scalar", "relu_", "copy_", "fill_.Scalar",
                "zero_", "bernoulli_.float")


class _MixedDtypeConv(TorchFunctionMode):
    """``F.conv2d`` refuses a bf16 input with an fp32 bias before dispatch (the fp32 master bias of SE
    gates / classifier convs): route such calls straight to ``aten.convolution``, whose native impl
    reads each operand in its own dtype."""

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is F.conv2d or func is torch.conv2d:
            a = list(args) + [None] * (7 - len(args))
            x, w, b = a[0], a[1], a[2] if len(args) > 2 else kwargs.get("bias")
            if (isinstance(x, torch.Tensor) and x.is_cuda and b is not None and b.dtype != x.dtype
                    and not isinstance(kwargs.get("padding", a[4]), str)):
                stride = kwargs.get("stride", a[3] if a[3] is not None else 1)
                padding = kwargs.get("padding", a[4] if a[4] is not None else 0)
                dilation = kwargs.get("dilation", a[5] if a[5] is not None else 1)
                groups = kwargs.get("groups", a[6] if a[6] is not None else 1)
                return aten.convolution.default(x, w, b, list(_pair(stride)), list(_pair(padding)),
                                                list(_pair(dilation)), False, [0, 0], int(groups))
        return func(*args, **kwargs)


class NativeMode(TorchDispatchMode):
    """Route a training step's aten ops to fedmi's HIP kernels (see module docstring)."""

    current: "NativeMode" = None

    def __init__(self, strict: bool = False, seed: int = 0, fuse: bool = True, discard_unread: bool = False):
        super().__init__()
        self.strict = strict
        # at exit, tensors a fused op left unwritten (deferred: nothing inside the block read them) are
        # materialised, because code after the block may still read them (e.g. a gradient AccumulateGrad adopted
        # as p.grad without dispatching an op).  A caller that provably reads nothing after the block (the
        # trainer: it copies every p.grad inside the block) sets discard_unread and saves those launches.
        self.discard_unread = bool(discard_unread)
        self.seed = seed
        self.fallbacks = collections.Counter()
        self.native_ops = collections.Counter()
        self._ctr = {}
        self.fuse = bool(fuse)          # BN -> ReLU (forward) and ReLU-backward -> BN-backward fusion
        self._pend_bn: Optional[_PendingBN] = None
        self._pend_thr: Optional[_PendingThr] = None
        self._dead = {}                 # storage ptr -> materialiser of a tensor a fused op never wrote
        self.fused = collections.Counter()
        self.packs = collections.Counter()   # weight images packed by the batched per-block launches
        self.scalar_ew = collections.Counter()   # (op, shape, strides) of elementwise passes on the scalar kernel
        self.ew_ops = collections.Counter()      # (aten op, elementwise op code) -> passes
        self.diag = False                        # collect scalar_ew / ew_ops (tools/prof_native_mode.py)
        self._wcache = {}               # packed conv weights of the current block (see _packed)
        self._pend_ctr: Optional[torch.Tensor] = None   # a BN counter increment waiting for its BN forward
        self._pend_bnb: Optional[_PendingBNB] = None    # a BN input gradient waiting for its accumulation add
        self._pend_mul: Optional[_PendingMul] = None    # a product waiting for the reduction that sums it
        self._pend_sb = {}              # storage ptr -> _PendingSliceBwd (deferred; see _sb_pair)
        self.stable_storage = 0         # data_ptr of the trainer's flat parameter storage (set by the trainer)
        self._pack_plan, self._wd_plan = {}, {}   # weight-image keys of stable weights -> fp32 master (kept)
        self.grad_flat: Optional[torch.Tensor] = None   # the trainer's flat gradient buffer (see _param_grad)
        self.bias_of = {}               # weight storage offset -> (bias offset, numel) of the same module
        self._grad_taken = set()
        self._prepacked = self._prepacked_wd = False
        self._cat_plan = {}             # concat-chain head shapes -> final width (kept across blocks)
        self._catbufs = {}              # storage ptr -> _CatBuf of the current block
        self._cat_src = {}              # (ptr, shape) of a plain cat output of this block -> its chain head
        # deferred WGRAD reductions (see _wred_part): FEDMI_WRED_DEFER=0 reduces each right away (A/B)
        self.defer_wred = os.environ.get("FEDMI_WRED_DEFER", "1") != "0"
        self._wred, self._wred_keep, self._wred_ptrs = [], [], set()

    def _defer(self, t: torch.Tensor, materialize) -> None:
        self._dead[t.untyped_storage().data_ptr()] = materialize

    def _prepack(self, wd: bool) -> None:
        """Pack every remembered weight image (``wd``: DGRAD images) of the trainer's parameters in as few
        launches as the multi-tensor pack kernels take (see :func:`_packed`)."""
        plan = self._wd_plan if wd else self._pack_plan
        items = []
        for key, w32 in plan.items():
            O8, C8, st, pd, groups = key[3:]
            ent = self._wcache.setdefault(key, (w32, {}))[1]
            if wd:
                if "wd" not in ent and w32.shape[0] == O8 and w32.is_contiguous() and groups == 1:
                    ent["wd"] = _wd_image(w32, O8, C8, st, pd)
                    items.append((w32, ent["wd"], st, pd, C8))
            elif "wp" not in ent and w32.is_contiguous():
                O, _, R, S = w32.shape
                ent["wp"] = torch.empty(O8, R, S, C8, dtype=torch.bfloat16, device=w32.device)
                items.append((w32, ent["wp"], groups))
        if items:
            (CV.dgrad_pack_weights if wd else CV.pack_weights)(items)
            self.packs["wd" if wd else "wp"] += len(items)

    def _flush_ctr(self) -> None:
        if self._pend_ctr is not None:
            t, self._pend_ctr = self._pend_ctr, None
            ew(t, [t], EW_ADDS, 1.0)

    def _take_ctr(self) -> Optional[torch.Tensor]:
        t, self._pend_ctr = self._pend_ctr, None
        return t

    def _flush_wred(self) -> None:
        if self._wred:
            items, self._wred = self._wred, []
            CV.wgrad_reduce_multi(items, self._wred_keep[0].device)
        self._wred_keep, self._wred_ptrs = [], set()

    def _flush(self) -> None:
        self._flush_wred()
        self._flush_ctr()
        if self._pend_mul is not None:
            pend, self._pend_mul = self._pend_mul, None
            pend.materialize()
        if self._pend_bnb is not None:
            pend, self._pend_bnb = self._pend_bnb, None
            pend.materialize()
        if self._pend_bn is not None:
            pend, self._pend_bn = self._pend_bn, None
            pend.materialize()
        if self._pend_thr is not None:
            pend, self._pend_thr = self._pend_thr, None
            pend.materialize()

    def _touch(self, args, kwargs) -> None:
        """Before an op runs: materialise a pending result it does not fuse with, and any deferred tensor
        it reads (a fused op left it unwritten)."""
        if self._pend_ctr is not None and self._func not in _BN_FWD:
            self._flush_ctr()
        if self._pend_mul is not None and not (self._func in (aten.sum.dim_IntList, aten.mean.dim) and args
                                               and _same(args[0], self._pend_mul.out)):
            pend, self._pend_mul = self._pend_mul, None
            pend.materialize()
        if self._pend_bnb is not None and not (self._func in (aten.add.Tensor, aten.add_.Tensor)
                                               and _bnb_add_partner(self._pend_bnb, args, kwargs) is not None):
            pend, self._pend_bnb = self._pend_bnb, None
            pend.materialize()
        if self._pend_bn is not None and not self._fuses_bn(args, kwargs):
            pend, self._pend_bn = self._pend_bn, None
            pend.materialize()
        if self._pend_thr is not None and not self._fuses_thr(args):
            pend, self._pend_thr = self._pend_thr, None
            pend.materialize()
        if self._wred_ptrs and any(t.data_ptr() in self._wred_ptrs for t in _iter_tensors(args, kwargs)):
            self._flush_wred()              # an op reads a weight gradient whose reduction is still pending
        if self._dead and self._pend_sb and self._func is aten.add.Tensor and _sb_pair(self, args, kwargs):
            return                          # the add reads both pending slice gradients' sources itself
        if self._dead:
            for t in _iter_tensors(args, kwargs):
                fn = self._dead.pop(t.untyped_storage().data_ptr(), None) if t.is_cuda else None
                if fn is not None:
                    fn()

    _func = None

    def _func_name(self) -> str:
        return str(self._func).replace("aten.", "") if self._func is not None else "?"

    def _fuses_bn(self, args, kwargs=None) -> bool:
        if self._func is aten.add.Tensor:
            return _bn_add_partner(self._pend_bn, args, kwargs) is not None
        return (self._func in (aten.relu.default, aten.relu_.default) and len(args) > 0
                and _same(args[0], self._pend_bn.out))

    def _fuses_thr(self, args) -> bool:
        if self._func is aten.native_batch_norm_backward.default:
            g = args[0] if args else None
        elif self._func is aten.miopen_batch_norm_backward.default:
            g = args[1] if len(args) > 1 else None
        else:
            return False
        return _same(g, self._pend_thr.out)

    def rng_ctr(self, dev) -> torch.Tensor:
        dev = torch.device(dev)
        if dev not in self._ctr:
            self._ctr[dev] = torch.zeros(4, dtype=torch.int32, device=dev)
        return self._ctr[dev]

    def __enter__(self):
        self._prev = NativeMode.current
        NativeMode.current = self
        self._wcache = {}
        self._pend_sb = {}
        self._prepacked = self._prepacked_wd = False
        self._catbufs, self._cat_src = {}, {}
        self._grad_taken = set()
        self._fn_mode = _MixedDtypeConv()
        self._fn_mode.__enter__()
        return super().__enter__()

    def __exit__(self, *exc):
        try:
            self._flush()
            if not self.discard_unread and exc[0] is None:
                for fn in list(self._dead.values()):
                    fn()
        finally:
            self._dead.clear()
            self._pend_sb = {}
            self._wcache = {}
            self._catbufs, self._cat_src = {}, {}
        NativeMode.current = self._prev
        try:
            return super().__exit__(*exc)
        finally:
            self._fn_mode.__exit__(*exc)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in _PASSTHROUGH:
            if func is aten._local_scalar_dense.default:     # reads device data: everything must be written
                self._flush()
                self._touch(args, kwargs)
            return func(*args, **kwargs)
        self._func = func
        if self._catbufs and func in _INPLACE and isinstance(args[0], torch.Tensor) and args[0].is_cuda \
                and args[0].untyped_storage().data_ptr() in self._catbufs:
            raise RuntimeError(f"native_mode: {func} writes in place into a shared concat buffer (a cat output "
                               "aliases the inputs of later cats); run this model with NativeMode(fuse=False)")
        self._touch(args, kwargs)
        fn = _IMPL.get(func)
        on_gpu = _dev(args, tuple(kwargs.values())) is not None
        if fn is not None and on_gpu:
            out = fn(func, *args, **kwargs)
            if out is ATEN:
                return func(*args, **kwargs)
            if out is not None:
                self.native_ops[str(func)] += 1
                return out
        if on_gpu:
            if self.strict:
                raise RuntimeError(f"native_mode: no native kernel for {func}")
            if not self.fallbacks[str(func)]:   # never silent: once per op, counted in .fallbacks (bench JSON)
                print(f"[fedmi native_mode] ATen fallback for {func} (FEDMI_NATIVE_STRICT=1 makes it an error)",
                      file=sys.stderr, flush=True)
            self.fallbacks[str(func)] += 1
        return func(*args, **kwargs)


def _iter_tensors(args, kwargs):
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor):
            yield a
        elif isinstance(a, (list, tuple)):
            for b in a:
                if isinstance(b, torch.Tensor):
                    yield b


def ce_stats_(logits: torch.Tensor, labels: torch.Tensor, stats: torch.Tensor) -> None:
    """stats (fp32 [3]) += (cross-entropy sum, correct, count) of a classifier batch (one native launch)."""
    y = labels if labels.dtype == torch.int64 else labels.long()
    _nat().z_ce_stats(_st(logits.device), zd(logits), y.data_ptr(), stats.data_ptr())


__all__ = ["NativeMode", "ce_stats_", "ew", "fill_", "reduce_sum", "zd"]
