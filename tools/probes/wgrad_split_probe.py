"""Probe: the generic split-K WGRAD (conv_igemm<WGRAD> + reduce) of GoogLeNet / DenseNet / MobileNet 1x1 and
narrow 3x3 convs at batch 128 -- automatic split count vs forced counts.  Graph-replayed µs per call (WGRAD +
reduce), the split count the launcher picked, and the operand-bandwidth floor (X + dY read once at 5 TB/s).

    python tools/probes/wgrad_split_probe.py
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402

from fedmi.ops import conv  # noqa: E402
from wgrad_gemm_probe import timed  # noqa: E402

# (N, H, C, O, R): GoogLeNet a3 / a4 / b5 1x1s, a3 16 -> 32 3x3, DenseNet 1x1 / 3x3, MobileNet 32x32 / 16x16 pointwise
SHAPES = [(128, 32, 192, 64, 1), (128, 32, 192, 96, 1), (128, 32, 256, 128, 1), (128, 16, 480, 192, 1),
          (128, 16, 512, 160, 1), (128, 8, 832, 256, 1), (128, 32, 16, 32, 3), (128, 16, 96, 208, 3),
          (128, 32, 96, 128, 1), (128, 32, 128, 32, 3), (128, 32, 32, 64, 1), (128, 16, 64, 128, 1)]


def main():
    dev = torch.device("cuda:0")
    for N, H, C, O, R in SHAPES:
        pad = R // 2
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        dy = torch.randn(N, H, H, O, device=dev).bfloat16()
        shp = (x.shape, O, R, R, 1, pad, C)
        auto_floats = conv.wgrad_ws_floats(*shp)
        plane = O * R * R * C
        ws = torch.empty(max(auto_floats, 1024 * plane), device=dev)
        dw = torch.empty(O, C, R, R, device=dev)
        row = {"N": N, "H": H, "C": C, "O": O, "R": R, "auto_splits": auto_floats // plane,
               "floor_us": round((x.numel() + dy.numel()) * 2 / 5e12 * 1e6, 2)}
        ref = None
        for sp in (0, 16, 32, 64, 128, 256, 512):
            ws_use = ws[:auto_floats] if sp == 0 else ws

            def run():
                conv.conv2d_wgrad(x, dy, R, R, 1, pad, Cw=C, out=dw, ws=ws_use, splits=sp, lib_gemm=False)
            try:
                row[f"us_{sp or 'auto'}"] = round(timed(run), 2)
                torch.cuda.synchronize()
                if ref is None:
                    ref = dw.clone()
                else:
                    row[f"rel_{sp}"] = float((dw - ref).abs().max() / ref.abs().max())
            except Exception as e:  # noqa: BLE001
                row[f"us_{sp}"] = repr(e)[:80]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
