"""Implicit-GEMM convolution on MFMA (csrc/kernels/conv_igemm.hip), NHWC bf16.

Functional wrappers over the native launches: they allocate outputs, check
shapes on the host (a kernel never sees an operand that disagrees with its
grid) and launch on torch's current stream.  Activations are channels-last
``[N, H, W, C]`` bf16 with ``C % 8 == 0`` (the network input is padded from 3
to 8 channels by :func:`fedmi.ops.cnn.prep_input`); weights are packed from the
fp32 PyTorch master ``[O, Cw, R, S]`` into ``[O, R, S, C]`` bf16.

Reference ops: ``convolution`` / ``convolution_backward`` of every zoo model
(e.g. src/models/resnet.py:14-70).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from .. import native


# BatchNorm statistics buffers are [STAT_REP, 2, C] fp64 replicas (csrc/kernels/common.h STAT_REP): the
# conv / depthwise epilogues add their fp32 workgroup partials into replica (workgroup % STAT_REP) with fp64
# atomics -- the totals do not depend on the order the workgroups arrive in (up to fp64 rounding, far
# below the fp32 mean / variance derived from them) -- and bn_apply sums the replicas in fixed order.
STAT_REP = 16


def stats_buffer(C: int, device) -> torch.Tensor:
    return torch.zeros(STAT_REP, 2, C, dtype=torch.float64, device=device)


def stats_total(stats: torch.Tensor) -> torch.Tensor:
    """[2, C] fp32 totals (sum, sum of squares) of a replicated fp64 statistics buffer."""
    return stats.view(STAT_REP, 2, -1).sum(0).float()


def _check_stats(stats: Optional[torch.Tensor], C: int, who: str) -> None:
    if stats is not None and (stats.numel() != STAT_REP * 2 * C or stats.dtype != torch.float64
                              or not stats.is_contiguous()):
        raise ValueError(f"{who}: stats must be contiguous fp64 [STAT_REP={STAT_REP}, 2, {C}]")


def pad8(c: int) -> int:
    return (c + 7) // 8 * 8


def out_hw(h: int, w: int, r: int, s: int, stride: int, pad: int) -> Tuple[int, int]:
    return (h + 2 * pad - r) // stride + 1, (w + 2 * pad - s) // stride + 1


def shape_tuple(x_shape, O: int, R: int, S: int, stride: int, pad: int, Cw: Optional[int] = None):
    """(N, H, W, C, Cw, O, P, Q, R, S, stride, pad) as the native launchers expect."""
    N, H, W, C = (int(v) for v in x_shape)
    P, Q = out_hw(H, W, R, S, stride, pad)
    if C % 8 or O % 8:
        raise ValueError(f"conv: channels must be multiples of 8 (C={C}, O={O})")
    if stride not in (1, 2):
        raise ValueError("conv: stride 1 or 2")
    return (N, H, W, C, int(Cw if Cw is not None else C), int(O), P, Q, int(R), int(S), int(stride), int(pad))


def _check(t: torch.Tensor, dtype, name: str):
    if t.dtype != dtype or not t.is_cuda or not t.is_contiguous():
        raise ValueError(f"{name}: expected contiguous {dtype} CUDA tensor, got {t.dtype} {t.device}")


def pack_weight(w: torch.Tensor, c_pad: Optional[int] = None, out: Optional[torch.Tensor] = None,
                o_pad: Optional[int] = None, groups: int = 1) -> torch.Tensor:
    """fp32 [O, Cw, R, S] -> bf16 [O8, R, S, C] (C = Cw rounded up to 8, zero pad; ``o_pad`` = O8 >= O: zero
    filters O..O8 written by the same launch).  ``groups`` > 1: the block-diagonal dense image of a grouped conv
    (C = groups * Cw channels, filter o holds its group's Cw channels and zeros elsewhere)."""
    O, Cw, R, S = w.shape
    C = c_pad or pad8(Cw * groups)
    O8 = max(int(o_pad or O), O)
    if out is None:
        out = torch.empty(O8, R, S, C, dtype=torch.bfloat16, device=w.device)
    _check(w, torch.float32, "pack_weight.w")
    if tuple(out.shape) != (O8, R, S, C) or not out.is_contiguous():
        raise ValueError(f"pack_weight: image {tuple(out.shape)} vs {(O8, R, S, C)}")
    native.require().conv_pack(native.stream_handle(w.device), w.data_ptr(), out.data_ptr(), O, Cw, C, R * S, O8,
                               int(groups))
    return out


def pack_weights(items) -> None:
    """Pack many ``(w fp32 [O,Cw,R,S], out bf16 [O8,R,S,C][, groups])`` items in one multi-tensor launch (``O8 >
    O``: zero filters O..O8; groups > 1: block-diagonal image, see :func:`pack_weight`)."""
    items = [tuple(it) if len(it) == 3 else (it[0], it[1], 1) for it in items]
    if not items:
        return
    for w, out, _ in items:
        _check(w, torch.float32, "pack_weights.w")
        _check(out, torch.bfloat16, "pack_weights.out")
        if out.shape[0] < w.shape[0] or tuple(out.shape[1:3]) != tuple(w.shape[2:]) or out.shape[3] < w.shape[1]:
            raise ValueError(f"pack_weights: image {tuple(out.shape)} vs master {tuple(w.shape)}")
    dev = items[0][0].device
    native.require().conv_pack_multi(
        native.stream_handle(dev),
        [(w.data_ptr(), o.data_ptr(), w.shape[0], w.shape[1], o.shape[3], w.shape[2] * w.shape[3], o.shape[0], int(g))
         for w, o, g in items])


def fd_ws_floats(x_shape, O: int, R: int, S: int, stride: int, pad: int, Cw: Optional[int] = None) -> int:
    """Split-K workspace (fp32 elements) the forward + data-gradient launches of this conv can use."""
    return int(native.require().conv_fd_ws_floats(shape_tuple(x_shape, O, R, S, stride, pad, Cw)))


def _ws_args(ws: Optional[torch.Tensor]):
    return (ws.data_ptr(), ws.numel()) if ws is not None else (0, 0)


def conv2d_fwd(x: torch.Tensor, wrsc: torch.Tensor, stride: int, pad: int, Cw: Optional[int] = None,
               stats: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
               shift: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
               res: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y[N,P,Q,O] = conv(x[N,H,W,C]) (+ ``res`` [N,P,Q,O] bf16, fused into the epilogue: pre-activation
    residual blocks; needs C % 64 == 0); ``stats`` ([STAT_REP, 2, O] fp64, :func:`stats_buffer`) +=
    per-channel sum / sum of squares of (y - shift) (``shift``: [O] fp32 or None = 0).  ``ws`` (fp32): optional split-K workspace for
    deep-K / few-tile shapes (see :func:`fd_ws_floats`)."""
    _check(x, torch.bfloat16, "conv2d_fwd.x")
    _check(wrsc, torch.bfloat16, "conv2d_fwd.w")
    O, R, S, C = wrsc.shape
    if C != x.shape[3]:
        raise ValueError(f"conv2d_fwd: weight C={C} vs input C={x.shape[3]}")
    shp = shape_tuple(x.shape, O, R, S, stride, pad, Cw)
    N, P, Q = shp[0], shp[6], shp[7]
    if out is None:
        out = torch.empty(N, P, Q, O, dtype=torch.bfloat16, device=x.device)
    elif tuple(out.shape) != (N, P, Q, O):
        raise ValueError("conv2d_fwd: bad out shape")
    _check_stats(stats, O, "conv2d_fwd")
    if res is not None:
        _check(res, torch.bfloat16, "conv2d_fwd.res")
        if tuple(res.shape) != (N, P, Q, O) or C % 64:
            raise ValueError("conv2d_fwd: res must be [N,P,Q,O] and the input C % 64 == 0")
    native.require().conv_fwd(native.stream_handle(x.device), shp, x.data_ptr(), wrsc.data_ptr(), out.data_ptr(),
                              stats.data_ptr() if stats is not None else 0,
                              shift.data_ptr() if shift is not None else 0, *_ws_args(ws),
                              res.data_ptr() if res is not None else 0)
    return out


def dgrad_image_numel(w_shape, c_pad: Optional[int] = None) -> int:
    O, Cw, R, S = (int(v) for v in w_shape)
    return O * R * S * (c_pad or pad8(Cw))


# FEDMI_TAP_GEN=0: convs with C % 64 != 0 (forward) / O % 64 != 0 (stride-1 DGRAD) stay on the generic implicit
# GEMM (conv_igemm.hip tap_gen_enabled; A/B runs)
TAP_GEN = os.environ.get("FEDMI_TAP_GEN", "1") != "0"
DGRAD_GEN = TAP_GEN and os.environ.get("FEDMI_DGRAD_GEN", "1") != "0"     # the stride-1 GEN DGRAD only (A/B)


def dgrad_eligible(O: int, stride: Optional[int] = None) -> bool:
    """The tap-major DGRAD reads dY as its input operand (O input channels): O % 64 == 0, or, at stride 1 (one
    phase: a plain conv_tap problem), any O % 8 == 0 from 16 channels on ``conv_tap<GEN>`` (several taps per K
    step).  ``stride`` None: the stride-independent condition."""
    return O % 64 == 0 or (stride == 1 and DGRAD_GEN and O % 8 == 0 and O >= 16)


def dgrad_pack_weights(items) -> None:
    """DGRAD weight images for the tap-major kernel: ``(w fp32 [O,Cw,R,S], img bf16, stride, pad, c_pad)``
    per conv (the image is the flipped/transposed weight, one block per sub-pixel phase), one launch."""
    items = list(items)
    if not items:
        return
    rows = []
    for w, img, stride, pad, c_pad in items:
        _check(w, torch.float32, "dgrad_pack_weights.w")
        _check(img, torch.bfloat16, "dgrad_pack_weights.img")
        O, Cw, R, S = w.shape
        if img.numel() < dgrad_image_numel(w.shape, c_pad) or not dgrad_eligible(O, int(stride)):
            raise ValueError("dgrad_pack_weights: image too small or O not DGRAD-eligible at this stride")
        rows.append((w.data_ptr(), img.data_ptr(), O, Cw, c_pad, R, S, int(stride), int(pad)))
    native.require().dgrad_pack_multi(native.stream_handle(items[0][0].device), rows)


class SgdPack:
    """One launch per step for a flat fp32 master: torch.optim.SGD on every element (bit-identical to
    ``sgd_flat``) and, for each dense conv, its forward image (:func:`pack_weights`) and DGRAD image
    (:func:`dgrad_pack_weights`) written from the updated values (``sgd_pack_kernel``).  The unfused tail reads
    the fp32 weights three times in 3-4 launches.

    ``convs``: ``(w, wr, wd, stride, pad, C)`` per conv -- ``w`` a view of ``params`` (the fp32 master [O, Cw, R, S]),
    ``wr`` its bf16 [O, R, S, C] image or None, ``wd`` its DGRAD image or None.  ``grad`` / ``mom`` share
    ``params``' layout.  The device table holds raw pointers: every tensor here must outlive the plan."""

    def __init__(self, params: torch.Tensor, grad: torch.Tensor, mom: torch.Tensor, convs) -> None:
        for t, nm in ((params, "params"), (grad, "grad"), (mom, "mom")):
            _check(t, torch.float32, f"SgdPack.{nm}")
        n = params.numel()
        if grad.numel() != n or mom.numel() != n:
            raise ValueError("SgdPack: params / grad / mom sizes differ")
        base = params.data_ptr()
        rows, cover, keep = [], [], [params, grad, mom]
        for w, wr, wd, stride, pad, C in convs:
            O, Cw, R, S = (int(v) for v in w.shape)
            d = w.data_ptr() - base
            if not w.is_contiguous() or w.dtype != torch.float32 or d % 4 or d < 0 or d // 4 + w.numel() > n:
                raise ValueError("SgdPack: a conv weight is not a contiguous fp32 view of params")
            if wr is not None:
                _check(wr, torch.bfloat16, "SgdPack.wr")
                if tuple(wr.shape) != (O, R, S, int(C)):
                    raise ValueError(f"SgdPack: image {tuple(wr.shape)} vs {(O, R, S, int(C))}")
            if wd is not None:
                _check(wd, torch.bfloat16, "SgdPack.wd")
                if wd.numel() < dgrad_image_numel(w.shape, C) or not dgrad_eligible(O, int(stride)):
                    raise ValueError("SgdPack: DGRAD image too small or O not DGRAD-eligible at this stride")
            rows.append((d // 4, wr.data_ptr() if wr is not None else 0, wd.data_ptr() if wd is not None else 0,
                         O, Cw, int(C), R, S, int(stride), int(pad)))
            cover.append((d // 4, d // 4 + w.numel()))
            keep += [t for t in (wr, wd) if t is not None]
        segs, at = [], 0
        for a, b in sorted(cover):
            if a < at:
                raise ValueError("SgdPack: conv weights overlap")
            if a > at:
                segs.append((at, a - at))
            at = b
        if at < n:
            segs.append((at, n - at))
        tab, self.n_entries, self.n_blocks, self.lds = native.require().sgd_pack_plan(rows, segs)
        self.table = torch.frombuffer(bytearray(tab), dtype=torch.uint8).to(params.device)
        self._keep = keep
        self.n_convs, self.n_segs = len(rows), len(segs)

    def step(self, lr: float, momentum: float, weight_decay: float, dampening: float = 0.0,
             nesterov: bool = False, first: bool = False) -> None:
        p, g, b = self._keep[:3]
        native.require().sgd_pack(native.stream_handle(p.device), self.table.data_ptr(), self.n_entries,
                                  self.n_blocks, self.lds, p.data_ptr(), g.data_ptr(), b.data_ptr(), float(lr),
                                  float(momentum), float(weight_decay), float(dampening), int(nesterov), int(first))


def conv2d_dgrad(dy: torch.Tensor, wrsc: torch.Tensor, x_shape, stride: int, pad: int, Cw: Optional[int] = None,
                 out: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
                 wd: Optional[torch.Tensor] = None, accumulate: bool = False, add: Optional[torch.Tensor] = None,
                 bn_sums: Optional[dict] = None) -> torch.Tensor:
    """dx[N,H,W,C] from dy[N,P,Q,O].  ``wd``: the conv's DGRAD weight image (:func:`dgrad_pack_weights`)
    selects the tap-major LDS-DMA kernel (O % 64 == 0); without it the generic implicit GEMM runs.
    ``accumulate``: out += dx (one branch's share of a multi-branch block's input gradient).
    ``add``: out = dx + add (another incoming grad of the same tensor, e.g. the shortcut's).
    ``bn_sums`` (dict rep, reps, z, y, mean, inv [, zb, meanb, invb: a projection-shortcut BN that shares
    the incoming grad] [, msc with y=None: the ReLU mask is z * msc[0] + msc[1] > 0]): the BatchNorm that
    produced this conv's input gets
    its backward channel sums from the epilogue (chained replica layout, :func:`cnn.bn_bwd` presummed)
    -- ``add`` / ``bn_sums`` need :func:`dgrad_fusable`."""
    _check(dy, torch.bfloat16, "conv2d_dgrad.dy")
    O, R, S, C = wrsc.shape
    shp = shape_tuple(x_shape, O, R, S, stride, pad, Cw)
    if tuple(dy.shape) != (shp[0], shp[6], shp[7], O):
        raise ValueError(f"conv2d_dgrad: dy shape {tuple(dy.shape)} vs expected {(shp[0], shp[6], shp[7], O)}")
    if out is None:
        if accumulate:
            raise ValueError("conv2d_dgrad: accumulate needs out")
        out = torch.empty(*x_shape, dtype=torch.bfloat16, device=dy.device)
    if wd is not None:
        _check(wd, torch.bfloat16, "conv2d_dgrad.wd")
        if wd.numel() < O * R * S * C:
            raise ValueError("conv2d_dgrad: dgrad image too small")
    bs = _bn_sums_desc(bn_sums, out)
    if add is not None and add.shape != out.shape:
        raise ValueError("conv2d_dgrad: add must have the output's shape")
    native.require().conv_dgrad(native.stream_handle(dy.device), shp, dy.data_ptr(), wrsc.data_ptr(), out.data_ptr(),
                                *_ws_args(ws), wd.data_ptr() if wd is not None else 0, int(accumulate),
                                add.data_ptr() if add is not None else 0, bs)
    return out


def _bn_sums_desc(bn_sums: Optional[dict], out: torch.Tensor) -> Optional[dict]:
    """Device-pointer dict of a BN-sums descriptor (rep, reps, z, y[, zb, meanb, invb], mean, inv) whose
    tensors are compact and shaped like the DGRAD output ``out``."""
    if bn_sums is None:
        return None
    z, y, zb = bn_sums["z"], bn_sums.get("y"), bn_sums.get("zb")
    for t in (z, y, zb):
        if t is not None and (t.shape != out.shape or not t.is_contiguous() or t.dtype != torch.bfloat16):
            raise ValueError("dgrad: BN sums need compact bf16 z / y / zb of the output's shape")
    C = out.shape[-1]
    rep = bn_sums["rep"]
    if rep.dtype != torch.float64 or rep.numel() < 3 * C * int(bn_sums["reps"]):
        raise ValueError("dgrad: BN sums replicas must be fp64 [reps][3][C]")
    bs = dict(rep=rep.data_ptr(), reps=int(bn_sums["reps"]), z=z.data_ptr(), y=y.data_ptr() if y is not None else 0,
              mean=bn_sums["mean"].data_ptr(), inv=bn_sums["inv"].data_ptr())
    if zb is not None:
        bs.update(zb=zb.data_ptr(), meanb=bn_sums["meanb"].data_ptr(), invb=bn_sums["invb"].data_ptr())
    msc = bn_sums.get("msc")
    if msc is not None:   # ReLU mask from z: [2][C] scale / shift as the forward applied them (bn_apply co_out)
        if y is not None or msc.dtype != torch.float32 or msc.numel() < 2 * C:
            raise ValueError("dgrad: BN sums msc needs y=None and a float32 [2][C] buffer")
        bs.update(msc=msc.data_ptr(), msc_ld=C)
    return bs


def dgrad_fusable(x_shape, O: int, R: int, S: int, stride: int, pad: int, Cw: Optional[int] = None,
                  has_wd: bool = True) -> bool:
    """Whether :func:`conv2d_dgrad` of this shape takes ``add`` / ``bn_sums`` (tap path, no empty phase)."""
    return bool(native.require().conv_dgrad_fusable(shape_tuple(x_shape, O, R, S, stride, pad, Cw), int(has_wd)))


_WS: dict = {}


def wgrad_workspace(device, floats: int) -> torch.Tensor:
    """Per-device fp32 split-K workspace for conv2d_wgrad (grown outside graph capture only)."""
    dev = torch.device(device)
    ws = _WS.get(dev)
    if ws is None or ws.numel() < floats:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("conv2d_wgrad: workspace must be reserved before graph capture "
                               "(call wgrad_workspace(dev, wgrad_ws_floats(...)) first)")
        ws = torch.empty(max(floats, 1 << 20), dtype=torch.float32, device=dev)
        _WS[dev] = ws
    return ws


def wgrad_ws_floats(x_shape, O: int, R: int, S: int, stride: int, pad: int, Cw: Optional[int] = None) -> int:
    return int(native.require().conv_wgrad_ws_floats(shape_tuple(x_shape, O, R, S, stride, pad, Cw)))


# Pixel count (N*H*W) up to which a 1x1 / stride-1 WGRAD goes to the library GEMM; FEDMI_WGRAD_GEMM=0 keeps every
# WGRAD native (A/B switch).
WGRAD_GEMM_PIXELS = 2048 if os.environ.get("FEDMI_WGRAD_GEMM", "1") != "0" else 0


def conv2d_wgrad(x: torch.Tensor, dy: torch.Tensor, R: int, S: int, stride: int, pad: int, Cw: Optional[int] = None,
                 out: Optional[torch.Tensor] = None, accumulate: bool = False, splits: int = 0,
                 ws: Optional[torch.Tensor] = None, Ow: Optional[int] = None, groups: int = 1,
                 deferred: Optional[list] = None, lib_gemm: bool = True) -> torch.Tensor:
    """dW fp32 [O, Cw, R, S] (PyTorch layout).  ``accumulate`` adds into ``out`` instead of overwriting.
    ``deferred`` (a list): the split-K reduction is not launched but appended as a descriptor, for ONE
    :func:`wgrad_reduce_multi` launch after the backward pass -- ``ws`` must then stay untouched until that launch
    (``out`` is not written before it).  ``lib_gemm`` False: neither the library GEMM route (WGRAD_GEMM_PIXELS) nor
    the 1x1 halo-kernel route (the CNN engine's; the aten backend keeps the generic kernel).
    ``Ow`` < O: dy carries zero-padded filters; only the first Ow land in ``out`` ([Ow, Cw, R, S]).
    ``groups`` > 1: a grouped conv run densely (block-diagonal image): filter o keeps its group's Cw channels.

    Split-K partials go to a workspace (plain stores) and one reduce launch sums
    them into ``out`` — no fp32 atomics on the gradient.
    """
    _check(x, torch.bfloat16, "conv2d_wgrad.x")
    _check(dy, torch.bfloat16, "conv2d_wgrad.dy")
    O = dy.shape[3]
    shp = shape_tuple(x.shape, O, R, S, stride, pad, Cw)
    if tuple(dy.shape) != (shp[0], shp[6], shp[7], O):
        raise ValueError("conv2d_wgrad: dy shape mismatch")
    Ow = O if Ow is None else int(Ow)
    if not 0 < Ow <= O:
        raise ValueError("conv2d_wgrad: 0 < Ow <= O")
    if out is None:
        out = torch.empty(Ow, shp[4], R, S, dtype=torch.float32, device=x.device)
        accumulate = False
    if tuple(out.shape) != (Ow, shp[4], R, S) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("conv2d_wgrad: out must be contiguous fp32 [Ow, Cw, R, S]")
    if (lib_gemm and WGRAD_GEMM_PIXELS and R == 1 and S == 1 and stride == 1 and pad == 0 and groups == 1 and Ow == O
            and not accumulate and not splits and shp[4] == shp[3] and shp[0] * shp[1] * shp[2] <= WGRAD_GEMM_PIXELS):
        # 1x1 / stride 1 over at most 2048 pixels (MobileNet's 4x4 / 2x2 pointwise layers): a plain GEMM
        # dW[O, C] = dY^T X, where one library launch beats split-K + reduce (15.5-15.8 vs 17.3-20.1 us at 4x4,
        # 8.1-8.6 vs 21.8-28.5 us at 2x2; the native kernel wins from 8x8 up: profiles/r6_cnn/wgrad1x1.jsonl).
        # The library result is bit-stable run to run.
        C = shp[3]
        torch.mm(dy.view(-1, O).t(), x.view(-1, C), out_dtype=torch.float32, out=out.view(O, C))
        return out
    nat = native.require()
    if deferred is not None and ws is None:
        raise ValueError("conv2d_wgrad: a deferred reduction needs its own workspace")
    if ws is None:
        need = max(nat.conv_wgrad_ws_floats(shp), splits * O * R * S * shp[3])
        ws = wgrad_workspace(x.device, need)
    item = nat.conv_wgrad(native.stream_handle(x.device), shp, x.data_ptr(), dy.data_ptr(), out.data_ptr(),
                          ws.data_ptr(), ws.numel(), splits, int(accumulate), Ow, int(groups), int(deferred is not None),
                          int(lib_gemm))
    if item is not None:
        deferred.append(item)
    return out


def wgrad_reduce_multi(items: list, device) -> None:
    """Run the WGRAD partial reductions collected by ``conv2d_wgrad`` / ``dwconv_wgrad`` (``deferred=``) in one
    launch (per 32 items); each item sums exactly as its immediate reduction would (bit-identical)."""
    if items:
        native.require().wgrad_reduce_multi(native.stream_handle(device), list(items))


# ---------------------------------------------------------------------------
# Depthwise convolution (csrc/kernels/dwconv.hip): groups == channels, weights
# used directly in the PyTorch fp32 layout [C, 1, R, S].
def _dw_shape(x_shape, R: int, stride: int, pad: int):
    N, H, W, C = (int(v) for v in x_shape)
    if C % 8 or C > 2048:
        raise ValueError(f"dwconv: C={C} must be a multiple of 8 and <= 2048")
    return (N, H, W, C, int(R), int(R), int(stride), int(pad))


def dwconv_fwd(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int, stats: Optional[torch.Tensor] = None,
               out: Optional[torch.Tensor] = None, shift: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Depthwise conv (NHWC bf16), fp32 weights [C, 1, R, R]; optional fused BN statistics of the output."""
    _check(x, torch.bfloat16, "dwconv_fwd.x")
    _check(w, torch.float32, "dwconv_fwd.w")
    C, one, R, S = w.shape
    if one != 1 or C != x.shape[3] or R != S:
        raise ValueError("dwconv_fwd: weight must be [C, 1, R, R]")
    shp = _dw_shape(x.shape, R, stride, pad)
    _check_stats(stats, C, "dwconv_fwd")
    P, Q = out_hw(shp[1], shp[2], R, R, stride, pad)
    if out is None:
        out = torch.empty(shp[0], P, Q, C, dtype=torch.bfloat16, device=x.device)
    native.require().dw_fwd(native.stream_handle(x.device), shp, x.data_ptr(), w.data_ptr(), out.data_ptr(),
                            stats.data_ptr() if stats is not None else 0,
                            shift.data_ptr() if shift is not None else 0)
    return out


def dwconv_dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape, stride: int, pad: int,
                 out: Optional[torch.Tensor] = None, bn_sums: Optional[dict] = None) -> torch.Tensor:
    """``bn_sums``: as :func:`conv2d_dgrad` (the producer BN's backward sums from the stored dx)."""
    _check(dy, torch.bfloat16, "dwconv_dgrad.dy")
    shp = _dw_shape(x_shape, w.shape[2], stride, pad)
    if out is None:
        out = torch.empty(*x_shape, dtype=torch.bfloat16, device=dy.device)
    native.require().dw_dgrad(native.stream_handle(dy.device), shp, dy.data_ptr(), w.data_ptr(), out.data_ptr(),
                              _bn_sums_desc(bn_sums, out))
    return out


def dwconv_ws_floats(x_shape, R: int, stride: int, pad: int) -> int:
    return int(native.require().dw_wgrad_ws_floats(_dw_shape(x_shape, R, stride, pad)))


def dwconv_wgrad(x: torch.Tensor, dy: torch.Tensor, R: int, stride: int, pad: int, out: Optional[torch.Tensor] = None,
                 accumulate: bool = False, ws: Optional[torch.Tensor] = None,
                 deferred: Optional[list] = None) -> torch.Tensor:
    """Depthwise dW fp32 [C, 1, R, R]; ``deferred``: as :func:`conv2d_wgrad`."""
    _check(x, torch.bfloat16, "dwconv_wgrad.x")
    _check(dy, torch.bfloat16, "dwconv_wgrad.dy")
    shp = _dw_shape(x.shape, R, stride, pad)
    C = shp[3]
    if out is None:
        out = torch.empty(C, 1, R, R, dtype=torch.float32, device=x.device)
        accumulate = False
    nat = native.require()
    if deferred is not None and ws is None:
        raise ValueError("dwconv_wgrad: a deferred reduction needs its own workspace")
    if ws is None:
        ws = wgrad_workspace(x.device, nat.dw_wgrad_ws_floats(shp))
    item = nat.dw_wgrad(native.stream_handle(x.device), shp, x.data_ptr(), dy.data_ptr(), out.data_ptr(),
                        ws.data_ptr(), ws.numel(), int(accumulate), int(deferred is not None))
    if item is not None:
        deferred.append(item)
    return out
