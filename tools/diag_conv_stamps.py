#!/usr/bin/env python
"""Per-phase cycles of conv_tap (diagnostic stamps build, FEDMI_NATIVE_VARIANT=stamps): prologue (offsets + DMA
issue), first-data wait, K loop (first half / second half), epilogue; median / max over workgroups.

    FEDMI_NATIVE_VARIANT=stamps python tools/diag_conv_stamps.py [--shapes l1,l2,l3,l4] [--pass fwd|dgrad]
"""
import argparse
import os
import sys
from pathlib import Path

os.environ.setdefault("FEDMI_NATIVE_VARIANT", "stamps")
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fedmi import native  # noqa: E402
from fedmi.ops import conv  # noqa: E402

SHAPES = {"l1": (32, 64, 64), "l2": (16, 128, 128), "l3": (8, 256, 256), "l4": (4, 512, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="l1,l2,l3,l4")
    ap.add_argument("--split", action="store_true", help="allow split-K (workspace)")
    a = ap.parse_args()
    nat = native.require()
    assert nat.stamps_enabled(), "not the stamps build"
    dev = torch.device("cuda", 0)
    for key in a.shapes.split(","):
        H, Ci, Co = SHAPES[key]
        x = (torch.randn(128, H, H, Ci, device=dev) * 0.5).bfloat16()
        w = torch.randn(Co, Ci, 3, 3, device=dev) * 0.05
        wr = conv.pack_weight(w)
        y = torch.empty(128, H, H, Co, dtype=torch.bfloat16, device=dev)
        ws = torch.empty(max(conv.fd_ws_floats(x.shape, Co, 3, 3, 1, 1, Ci), 1), device=dev) if a.split else None
        for _ in range(20):
            conv.conv2d_fwd(x, wr, 1, 1, Cw=Ci, out=y, ws=ws)
        torch.cuda.synchronize()
        nat.read_conv_stamps(True)
        conv.conv2d_fwd(x, wr, 1, 1, Cw=Ci, out=y, ws=ws)
        torch.cuda.synchronize()
        st = np.frombuffer(nat.read_conv_stamps(True), dtype=np.uint64).reshape(nat.STAMP_SHAPE[1:]).astype(np.int64)
        rows = st[(st[:, 0] > 0) & (st[:, 5] > 0)]
        d = np.diff(rows[:, :6], axis=1)
        # s_memtime is a per-XCD counter: differences within one workgroup are meaningful, absolute values
        # across workgroups (start/end spread) are not, so only per-WG phase lengths are reported
        print(f"{key}: wgs {len(rows)}  total med {np.median(rows[:, 5] - rows[:, 0]):.0f}")
        for j, ph in enumerate(["offsets+DMA issue", "first data", "loop 1st half", "loop 2nd half", "epilogue"]):
            print(f"    {ph:18s} med {np.median(d[:, j]):8.0f}  max {d[:, j].max():8.0f}")


if __name__ == "__main__":
    main()
