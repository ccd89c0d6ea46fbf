#!/usr/bin/env python
"""Time the conv kernels on chosen ResNet-18 batch-128 shapes with variants
(tap FWD with / without BN stats, tap DGRAD, generic WGRAD), for rocprofv3 PMC
passes and quick A/B checks.

    python tools/bench_tap.py [--iters 50] [--shapes l1,l2,l3,l4]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from fedmi.ops import conv  # noqa: E402

SHAPES = {"l1": (32, 64, 64, 3, 1), "l2": (16, 128, 128, 3, 1), "l3": (8, 256, 256, 3, 1), "l4": (4, 512, 512, 3, 1),
          "d2": (32, 64, 128, 3, 2), "d4": (8, 256, 512, 3, 2)}


GRAPH = False


def timeit(fn, iters):
    """us per call; with --graph the calls are captured once and replayed (no host launch cost)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    if GRAPH:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        run = g.replay
    else:
        def run():
            for _ in range(iters):
                fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default="l1,l2,l3,l4,d2,d4")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--graph", action="store_true", help="time graph replays (kernel time, no launch cost)")
    ap.add_argument("--passes", default="", help="comma list of passes to run (default: all)")
    a = ap.parse_args()
    global GRAPH
    GRAPH = a.graph
    dev = torch.device("cuda", 0)
    N = a.batch
    for key in a.shapes.split(","):
        H, Ci, Co, k, st = SHAPES[key]
        pad = k // 2
        x = (torch.randn(N, H, H, Ci, device=dev) * 0.5).bfloat16()
        w = torch.randn(Co, Ci, k, k, device=dev) * 0.05
        wr = conv.pack_weight(w)
        wd = torch.empty(conv.dgrad_image_numel(w.shape, Ci), dtype=torch.bfloat16, device=dev)
        conv.dgrad_pack_weights([(w, wd, st, pad, Ci)])
        P = (H + 2 * pad - k) // st + 1
        dy = (torch.randn(N, P, P, Co, device=dev) * 0.5).bfloat16()
        y = torch.empty(N, P, P, Co, dtype=torch.bfloat16, device=dev)
        dx = torch.empty_like(x)
        dw = torch.zeros(Co, Ci, k, k, device=dev)
        stats = conv.stats_buffer(Co, dev)
        shp = (x.shape, Co, k, k, st, pad, Ci)
        ws = torch.empty(max(conv.fd_ws_floats(*shp), conv.wgrad_ws_floats(*shp), 1), device=dev)
        flops = 2.0 * N * P * P * Co * Ci * k * k
        runs = {
            "fwd_stats": lambda: conv.conv2d_fwd(x, wr, st, pad, Cw=Ci, stats=stats, out=y, ws=ws),
            "fwd_nostats": lambda: conv.conv2d_fwd(x, wr, st, pad, Cw=Ci, out=y, ws=ws),
            "fwd_nosplit": lambda: conv.conv2d_fwd(x, wr, st, pad, Cw=Ci, stats=stats, out=y),
            "dgrad_tap": lambda: conv.conv2d_dgrad(dy, wr, x.shape, st, pad, Cw=Ci, out=dx, ws=ws, wd=wd),
            "dgrad_generic": lambda: conv.conv2d_dgrad(dy, wr, x.shape, st, pad, Cw=Ci, out=dx, ws=ws),
            "wgrad": lambda: conv.conv2d_wgrad(x, dy, k, k, st, pad, Cw=Ci, out=dw, ws=ws),
        }
        for name, fn in runs.items():
            if a.passes and name not in a.passes.split(","):
                continue
            us = timeit(fn, a.iters)
            print(json.dumps({"shape": key, "pass": name, "us": round(us, 2), "tflops": round(flops / us / 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
