"""Probe: 1x1 / stride-1 WGRAD per shape (batch 128, C and O % 64), graph-replayed µs per call (WGRAD + reduce) of
whatever route the launcher takes -- run twice, with FEDMI_WGRAD_1X1=0 (generic split-K conv_igemm) and =1
(conv_wgrad_halo<1, 1>), to pick the shapes the one-tap halo kernel should take.  ``--lib`` keeps the library GEMM
route of <= 2048-pixel problems (MobileNet's 4x4 / 2x2 pointwise convs) for the halo-vs-library comparison.

    FEDMI_WGRAD_1X1=1 python tools/probes/wgrad1x1_halo_probe.py [--lib]
"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402

from fedmi.ops import conv  # noqa: E402
from wgrad_gemm_probe import timed  # noqa: E402

# (H, C, O): MobileNet 16x16 / 8x8 pointwise, GoogLeNet 32x32 / 16x16 / 8x8 1x1 branches with C, O % 64
SHAPES = [(16, 64, 128), (16, 128, 128), (8, 128, 256), (8, 256, 256),
          (32, 192, 64), (32, 256, 128), (32, 256, 64), (16, 512, 128), (16, 512, 192), (16, 528, 256),
          (8, 832, 256), (8, 832, 384), (8, 832, 128),
          (4, 256, 512), (4, 512, 512), (2, 512, 1024), (2, 1024, 1024)]     # MobileNet 4x4 / 2x2 (library route)


def main():
    dev = torch.device("cuda:0")
    mode = os.environ.get("FEDMI_WGRAD_1X1", "1")
    lib = "--lib" in sys.argv
    if not lib:
        conv.WGRAD_GEMM_PIXELS = 0      # CNN-engine routing (lib_gemm=True) minus the small-M library GEMM
    for H, C, O in SHAPES:
        if C % 64 or O % 64:
            continue
        x = torch.randn(128, H, H, C, device=dev).bfloat16()
        dy = torch.randn(128, H, H, O, device=dev).bfloat16()
        shp = (x.shape, O, 1, 1, 1, 0, C)
        ws = torch.empty(max(conv.wgrad_ws_floats(*shp), 1), device=dev)
        dw = torch.empty(O, C, 1, 1, device=dev)

        def run():
            conv.conv2d_wgrad(x, dy, 1, 1, 1, 0, out=dw, ws=ws)
        print(json.dumps({"H": H, "C": C, "O": O, "halo1": mode, "lib": lib, "us": round(timed(run), 2),
                          "splits": ws.numel() // (O * C)}), flush=True)


if __name__ == "__main__":
    main()
