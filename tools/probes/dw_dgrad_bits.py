"""Probe: the blocked depthwise DGRAD kernels vs the per-pixel kernel they replace, bit for bit.

    python tools/probes/dw_dgrad_bits.py --save-old     (build with the per-pixel kernel dispatched)
    python tools/probes/dw_dgrad_bits.py                (build under test)

Writes / compares gpurun_out/dw_dgrad_old.pt.  Round 5 ran it with a temporary switch that dispatched the
per-pixel kernel (profiles/r5_cnn/experiments/bisect_efficientnet_dw_dgrad.txt: stride-2 shapes identical).
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from fedmi.ops import conv  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(3)
    outs = []
    for N, H, C, st in [(8, 32, 32, 1), (8, 16, 96, 2), (4, 9, 64, 2), (4, 7, 40, 1), (16, 8, 256, 1)]:
        P = (H + 2 - 3) // st + 1
        dy = torch.randn(N, P, P, C, generator=g).to(dev).bfloat16()
        w = (torch.randn(C, 1, 3, 3, generator=g) / 3).to(dev)
        outs.append(conv.dwconv_dgrad(dy, w, (N, H, H, C), st, 1).cpu())
    path = Path("gpurun_out/dw_dgrad_old.pt")
    if "--save-old" in sys.argv:
        path.parent.mkdir(exist_ok=True)
        torch.save(outs, path)
        print("saved", len(outs))
        return
    old = torch.load(path, weights_only=True)
    same = [bool(torch.equal(a, b)) for a, b in zip(outs, old)]
    print("bit-identical per shape:", same)
    sys.exit(0 if all(same) else 1)


if __name__ == "__main__":
    main()
