"""Native MFMA convolution as autograd layers, for zoo models without a whole-network engine.

The whole-network engines (``engine/cnn_native.py``) cover ResNet / PreActResNet / VGG / MobileNet /
MobileNetV2 / GoogLeNet.  The rest of the zoo (DenseNet, DLA, SENet, RegNet, ResNeXt, DPN,
ShuffleNetV2, EfficientNet, PNASNet) trains through PyTorch autograd; this module
puts the implicit-GEMM conv kernels (``csrc/kernels/conv_igemm.hip``: forward, data gradient,
weight gradient) under every eligible ``nn.Conv2d`` of such a model, with the activations kept
channels-last bf16 end to end (the network runs under bf16 autocast; BN / pooling / concat stay in
PyTorch on the same NHWC tensors, so no layout change happens between layers).

Eligible: ``groups == 1``, no dilation, stride 1 or 2 (square), symmetric zero padding, in/out channels
multiples of 8.  Grouped convs with at most 8 groups of width % 8 == 0 (ResNeXt) run one implicit
GEMM per group on channel-sliced copies.  Depthwise convs (``groups == C == O``, square 3/5/7 windows, C % 8 == 0, C <= 2048) run
on the depthwise kernels (``csrc/kernels/dwconv.hip``).  Every other conv (grouped, odd widths, the
3-channel stems) runs PyTorch's fp32 NCHW kernel: MIOpen's bf16 channels-last grouped / odd-width
convolutions measured up to 2x slower than its fp32 ones (profiles/hybrid_engine_r1.jsonl).
Weights stay the fp32 masters of the flat parameter buffer; each call packs them to the bf16
``[O, R, S, C]`` image (one small launch) and the weight gradient is produced in fp32 directly.

Reference ops replaced: ``convolution`` / ``convolution_backward`` of e.g. ``src/models/densenet.py:9-33``,
``src/models/dla.py:11-50``, ``src/models/senet.py:10-42``.
"""
from __future__ import annotations

import types
from typing import List

import torch
from torch import nn

from . import conv as C


def conv_eligible(m: nn.Module) -> bool:
    if type(m) is not nn.Conv2d:
        return False
    k, s, p, d = m.kernel_size, m.stride, m.padding, m.dilation
    return (m.groups == 1 and d == (1, 1) and s[0] == s[1] and s[0] in (1, 2) and not isinstance(p, str)
            and p[0] == p[1] and m.padding_mode == "zeros" and m.in_channels % 8 == 0
            and m.out_channels % 8 == 0 and k[0] <= 7 and k[1] <= 7)


MAX_GROUPS = 8


def grouped_eligible(m: nn.Module) -> bool:
    """Grouped conv with few, wide groups (ResNeXt cardinality <= 8, group width % 8 == 0): one MFMA
    implicit GEMM per group on channel-sliced copies of the operands."""
    if type(m) is not nn.Conv2d or not (1 < m.groups <= MAX_GROUPS):
        return False
    k, s, p, d = m.kernel_size, m.stride, m.padding, m.dilation
    G = m.groups
    return (m.in_channels % (8 * G) == 0 and m.out_channels % (8 * G) == 0 and d == (1, 1) and s[0] == s[1]
            and s[0] in (1, 2) and not isinstance(p, str) and p[0] == p[1] and m.padding_mode == "zeros"
            and k[0] <= 7 and k[1] <= 7)


def dw_eligible(m: nn.Module) -> bool:
    if type(m) is not nn.Conv2d:
        return False
    k, s, p, d = m.kernel_size, m.stride, m.padding, m.dilation
    C = m.in_channels
    return (m.groups == C == m.out_channels and C % 8 == 0 and C <= 2048 and k[0] == k[1] and k[0] in (3, 5, 7)
            and d == (1, 1) and s[0] == s[1] and s[0] in (1, 2) and not isinstance(p, str) and p[0] == p[1]
            and m.padding_mode == "zeros" and C * k[0] * k[1] * 4 <= 128 * 1024)


def fallback(m: nn.Module) -> bool:
    return type(m) is nn.Conv2d and not conv_eligible(m) and not dw_eligible(m) and not grouped_eligible(m)


def _nhwc_bf16(t: torch.Tensor) -> torch.Tensor:
    """NCHW-shaped tensor -> contiguous NHWC bf16 (a view when it already is channels-last bf16)."""
    return t.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()


def _ws(dev, floats: int):
    return C.wgrad_workspace(dev, floats) if floats > 0 else None


class _NativeConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride: int, pad: int):
        xh = _nhwc_bf16(x)
        O, Cw, R, S = w.shape
        wp = C.pack_weight(w.detach())
        ws = _ws(x.device, C.fd_ws_floats(xh.shape, O, R, S, stride, pad))
        y = C.conv2d_fwd(xh, wp, stride, pad, ws=ws)
        ctx.save_for_backward(xh, w, wp)
        ctx.stride, ctx.pad, ctx.x_dtype = stride, pad, x.dtype
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        xh, w, wp = ctx.saved_tensors
        stride, pad = ctx.stride, ctx.pad
        O, Cw, R, S = w.shape
        gyh = _nhwc_bf16(gy)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wd = None
            if C.dgrad_eligible(O):
                wd = torch.empty(C.dgrad_image_numel(w.shape), dtype=torch.bfloat16, device=w.device)
                C.dgrad_pack_weights([(w.detach(), wd, stride, pad, xh.shape[3])])
            ws = _ws(gy.device, C.fd_ws_floats(xh.shape, O, R, S, stride, pad))
            dx = C.conv2d_dgrad(gyh, wp, xh.shape, stride, pad, ws=ws, wd=wd).permute(0, 3, 1, 2)
            if ctx.x_dtype != torch.bfloat16:
                dx = dx.to(ctx.x_dtype)
        if ctx.needs_input_grad[1]:
            dw = C.conv2d_wgrad(xh, gyh, R, S, stride, pad)
        return dx, dw, None, None


class _NativeGroupedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride: int, pad: int, groups: int):
        xh = _nhwc_bf16(x)
        O, Cg, R, S = w.shape
        Og = O // groups
        xs, wps, ys = [], [], []
        for g in range(groups):
            xg = xh[..., g * Cg:(g + 1) * Cg].contiguous()
            wp = C.pack_weight(w.detach()[g * Og:(g + 1) * Og])
            ws = _ws(x.device, C.fd_ws_floats(xg.shape, Og, R, S, stride, pad))
            ys.append(C.conv2d_fwd(xg, wp, stride, pad, ws=ws))
            xs.append(xg)
            wps.append(wp)
        ctx.save_for_backward(w, *xs, *wps)
        ctx.stride, ctx.pad, ctx.groups, ctx.x_dtype = stride, pad, groups, x.dtype
        return torch.cat(ys, dim=3).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        G, stride, pad = ctx.groups, ctx.stride, ctx.pad
        w, xs, wps = ctx.saved_tensors[0], ctx.saved_tensors[1:1 + G], ctx.saved_tensors[1 + G:]
        O, Cg, R, S = w.shape
        Og = O // G
        gyh = _nhwc_bf16(gy)
        dxs, dws = [], []
        for g in range(G):
            dyg = gyh[..., g * Og:(g + 1) * Og].contiguous()
            if ctx.needs_input_grad[0]:
                ws = _ws(gy.device, C.fd_ws_floats(xs[g].shape, Og, R, S, stride, pad))
                dxs.append(C.conv2d_dgrad(dyg, wps[g], xs[g].shape, stride, pad, ws=ws))
            if ctx.needs_input_grad[1]:
                dws.append(C.conv2d_wgrad(xs[g], dyg, R, S, stride, pad))
        dx = dw = None
        if dxs:
            dx = torch.cat(dxs, dim=3).permute(0, 3, 1, 2)
            if ctx.x_dtype != torch.bfloat16:
                dx = dx.to(ctx.x_dtype)
        if dws:
            dw = torch.cat(dws, dim=0)
        return dx, dw, None, None, None


class _NativeDWFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride: int, pad: int):
        xh = _nhwc_bf16(x)
        y = C.dwconv_fwd(xh, w.detach(), stride, pad)
        ctx.save_for_backward(xh, w)
        ctx.stride, ctx.pad, ctx.x_dtype = stride, pad, x.dtype
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        xh, w = ctx.saved_tensors
        gyh = _nhwc_bf16(gy)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = C.dwconv_dgrad(gyh, w.detach(), xh.shape, ctx.stride, ctx.pad).permute(0, 3, 1, 2)
            if ctx.x_dtype != torch.bfloat16:
                dx = dx.to(ctx.x_dtype)
        if ctx.needs_input_grad[1]:
            dw = C.dwconv_wgrad(xh, gyh, w.shape[2], ctx.stride, ctx.pad)
        return dx, dw, None, None


def native_conv2d(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> torch.Tensor:
    """conv2d(x, w) on the MFMA kernels: x NCHW-shaped (best channels-last bf16), w fp32 [O, C, R, S].
    Returns NCHW-shaped bf16 in channels-last memory."""
    if x.shape[1] != w.shape[1]:
        raise ValueError(f"native_conv2d: input C={x.shape[1]} vs weight C={w.shape[1]}")
    if w.dtype != torch.float32 or not w.is_contiguous():
        raise ValueError("native_conv2d: weight must be the contiguous fp32 master")
    return _NativeConvFn.apply(x, w, int(stride), int(pad))


def _forward(self: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    if self.kernel_size == (1, 1) and x.shape[2] == 1 and x.shape[3] == 1:
        return _fallback_forward(self, x)       # squeeze-excite FC on a 1x1 map: a tiny fp32 GEMM
    y = native_conv2d(x, self.weight, self.stride[0], self.padding[0])
    if self.bias is not None:
        y = y + self.bias.to(y.dtype).view(1, -1, 1, 1)
    return y


def _dw_forward(self: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    if self.weight.dtype != torch.float32 or not self.weight.is_contiguous():
        raise ValueError("native depthwise conv: weight must be the contiguous fp32 master")
    y = _NativeDWFn.apply(x, self.weight, int(self.stride[0]), int(self.padding[0]))
    if self.bias is not None:
        y = y + self.bias.to(y.dtype).view(1, -1, 1, 1)
    return y


def _grouped_forward(self: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    if self.weight.dtype != torch.float32 or not self.weight.is_contiguous():
        raise ValueError("native grouped conv: weight must be the contiguous fp32 master")
    y = _NativeGroupedFn.apply(x, self.weight, int(self.stride[0]), int(self.padding[0]), int(self.groups))
    if self.bias is not None:
        y = y + self.bias.to(y.dtype).view(1, -1, 1, 1)
    return y


def _fallback_forward(self: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    if (self.kernel_size == (1, 1) and self.groups == 1 and self.padding in ((0, 0), 0) and x.shape[2] == 1
            and x.shape[3] == 1):
        # 1x1 conv on a 1x1 map (squeeze-excite FCs): a plain fp32 GEMM, no MIOpen solver search
        with torch.autocast("cuda", enabled=False):
            y = torch.nn.functional.linear(x.float().flatten(1), self.weight.flatten(1), self.bias)
        return y.to(torch.bfloat16)[:, :, None, None]
    with torch.autocast("cuda", enabled=False):
        y = nn.Conv2d._conv_forward(self, x.float().contiguous(), self.weight, self.bias)
    return y.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def install(model: nn.Module) -> List[str]:
    """Route every eligible ``nn.Conv2d`` of ``model`` through the native kernels (instance-level
    ``forward`` override: parameters, state-dict keys and module structure are untouched) and the
    remaining convs through PyTorch's fp32 NCHW kernel.  Returns the names of the native convs."""
    done = []
    for name, m in model.named_modules():
        if conv_eligible(m):
            m.forward = types.MethodType(_forward, m)
            done.append(name)
        elif dw_eligible(m):
            m.forward = types.MethodType(_dw_forward, m)
            done.append(name)
        elif grouped_eligible(m):
            m.forward = types.MethodType(_grouped_forward, m)
            done.append(name)
        elif fallback(m):
            m.forward = types.MethodType(_fallback_forward, m)
    return done


def coverage(model: nn.Module) -> dict:
    """{'native': n, 'fallback': n, 'native_weight_frac': f} over the model's Conv2d modules (MACs at 32x32
    are not known without a forward; the fraction counts weight elements as a proxy)."""
    nat = fb = 0
    wn = wt = 0
    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            k = m.weight.numel()
            wt += k
            if conv_eligible(m) or dw_eligible(m) or grouped_eligible(m):
                nat += 1
                wn += k
            else:
                fb += 1
    return {"native": nat, "fallback": fb, "native_weight_frac": (wn / wt) if wt else 0.0}


__all__ = ["conv_eligible", "grouped_eligible", "dw_eligible", "fallback", "native_conv2d", "install", "coverage"]
