"""Per-shape timing of the implicit-GEMM conv kernels vs PyTorch (MIOpen) at the
ResNet-18 CIFAR batch-128 shapes.  Prints one JSON line per
(shape, pass) with both times and our TFLOP/s.

    python tools/bench_conv.py [--batch 128] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from fedmi.ops import conv  # noqa: E402

# (H, Cin, Cout, k, stride) — input spatial size H=W
SHAPES = [(32, 3, 64, 3, 1), (32, 64, 64, 3, 1), (32, 64, 128, 3, 2), (32, 64, 128, 1, 2), (16, 128, 128, 3, 1),
          (16, 128, 256, 3, 2), (16, 128, 256, 1, 2), (8, 256, 256, 3, 1), (8, 256, 512, 3, 2), (8, 256, 512, 1, 2),
          (4, 512, 512, 3, 1)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N = a.batch
    tot = {"ours": 0.0, "torch": 0.0}
    for H, Ci, Co, k, st in SHAPES:
        pad = k // 2
        C = conv.pad8(Ci)
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        if C != Ci:
            x[..., Ci:] = 0
        w = torch.randn(Co, Ci, k, k, device=dev) * 0.05
        wr = conv.pack_weight(w)
        P = (H + 2 * pad - k) // st + 1
        dy = torch.randn(N, P, P, Co, device=dev).bfloat16()
        stats = conv.stats_buffer(Co, dev)
        y = torch.empty(N, P, P, Co, dtype=torch.bfloat16, device=dev)
        dx = torch.empty_like(x)
        dw = torch.zeros(Co, Ci, k, k, device=dev)
        # torch reference: channels_last bf16 (MIOpen)
        xt = x[..., :Ci].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        wt = w.bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
        dyt = dy.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        flops = 2.0 * N * P * P * Co * Ci * k * k
        ours = {
            "fwd": lambda: conv.conv2d_fwd(x, wr, st, pad, Cw=Ci, stats=stats, out=y),
            "dgrad": lambda: conv.conv2d_dgrad(dy, wr, x.shape, st, pad, Cw=Ci, out=dx),
            "wgrad": lambda: conv.conv2d_wgrad(x, dy, k, k, st, pad, Cw=Ci, out=dw),
        }
        ref = {
            "fwd": lambda: F.conv2d(xt, wt, stride=st, padding=pad),
            "dgrad": lambda: torch.ops.aten.convolution_backward(dyt, xt, wt, None, [st, st], [pad, pad], [1, 1],
                                                                 False, [0, 0], 1, [True, False, False]),
            "wgrad": lambda: torch.ops.aten.convolution_backward(dyt, xt, wt, None, [st, st], [pad, pad], [1, 1],
                                                                 False, [0, 0], 1, [False, True, False]),
        }
        for ph in ("fwd", "dgrad", "wgrad"):
            if ph == "dgrad" and Ci == 3:
                continue   # the stem's input grad is never needed
            t_o = timeit(ours[ph], a.iters)
            t_r = timeit(ref[ph], a.iters)
            tot["ours"] += t_o
            tot["torch"] += t_r
            print(json.dumps({"shape": [N, H, Ci, Co, k, st], "pass": ph, "ours_us": round(t_o, 1),
                              "torch_us": round(t_r, 1), "ours_tflops": round(flops / t_o / 1e6, 1),
                              "speedup": round(t_r / t_o, 2)}), flush=True)
    print(json.dumps({"total_ours_us": round(tot["ours"], 1), "total_torch_us": round(tot["torch"], 1)}))


if __name__ == "__main__":
    main()
