"""Probe: K-split count of the generic (split-K conv_igemm + reduce) weight gradient at ResNet-18's layer-4 shapes.

    python tools/probes/wgrad_splits_probe.py [--mobilenet]

Prints µs per conv2d_wgrad call (graph replay) for each split count; 0 = the automatic choice.
--mobilenet: MobileNet's 1x1 (pointwise) layers instead of ResNet-18's layer-4 shapes.
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from fedmi.ops import conv  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent))
from wgrad_gemm_probe import timed  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    # (N, H, C, O, R, stride, pad): l4 3x3, l4.0 3x3 stride 2, l4.0 1x1 shortcut, l3 1x1 shortcut
    shapes = [(128, 4, 512, 512, 3, 1, 1), (128, 8, 256, 512, 3, 2, 1), (128, 8, 256, 512, 1, 2, 0),
              (128, 16, 128, 256, 1, 2, 0)]
    if "--mobilenet" in sys.argv:
        shapes = [(128, 32, 32, 64, 1, 1, 0), (128, 16, 128, 128, 1, 1, 0), (128, 8, 256, 256, 1, 1, 0),
                  (128, 4, 256, 512, 1, 1, 0), (128, 4, 512, 512, 1, 1, 0), (128, 2, 512, 1024, 1, 1, 0),
                  (128, 2, 1024, 1024, 1, 1, 0)]
    for N, H, C, O, R, st, pad in shapes:
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        P = (H + 2 * pad - R) // st + 1
        dy = torch.randn(N, P, P, O, device=dev).bfloat16()
        shp = (x.shape, O, R, R, st, pad, C)
        dw = torch.empty(O, C, R, R, device=dev)
        ref = None
        row = {"N": N, "H": H, "C": C, "O": O, "R": R, "stride": st}
        for sp in ((0, 2, 4, 8, 16, 32) if "--mobilenet" in sys.argv else (0, 1, 2, 3, 4, 6, 8)):
            ws = torch.empty(max(conv.wgrad_ws_floats(*shp), max(sp, 1) * O * C * R * R, 1), device=dev)

            def run():
                conv.conv2d_wgrad(x, dy, R, R, st, pad, Cw=C, out=dw, ws=ws, splits=sp)

            row[f"sp{sp}_us"] = round(timed(run), 2)
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = dw.clone()
            else:
                row[f"sp{sp}_err"] = float((dw - ref).norm() / ref.norm())
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
