"""Phase timing of conv_halo from in-kernel s_memtime stamps (diagnostic build path, same binary):
prologue (start -> first step's data landed), main loop, epilogue, per workgroup; and the spread of
workgroup start times (s_memrealtime, 100 MHz).

    FEDMI_CONV_HALO=1 python tools/halo_stamps.py [--batch 128] [--shapes l1,l2,l3,l4]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from fedmi import native  # noqa: E402
from fedmi.ops import conv  # noqa: E402

SHAPES = {"l1": (32, 64, 64), "l2": (16, 128, 128), "l3": (8, 256, 256), "l4": (4, 512, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--shapes", default="l1,l2,l3,l4")
    ap.add_argument("--split", action="store_true", help="pass the split-K workspace")
    a = ap.parse_args()
    os.environ["FEDMI_CONV_HALO"] = "1"
    dev = torch.device("cuda", 0)
    nat = native.require()
    buf = torch.zeros(8 * 65536, dtype=torch.int64, device=dev)
    for key in a.shapes.split(","):
        H, Ci, Co = SHAPES[key]
        x = (torch.randn(a.batch, H, H, Ci, device=dev) * 0.5).bfloat16()
        wr = conv.pack_weight(torch.randn(Co, Ci, 3, 3, device=dev) * 0.05)
        y = torch.empty(a.batch, H, H, Co, dtype=torch.bfloat16, device=dev)
        stats = conv.stats_buffer(Co, dev)
        shp = (x.shape, Co, 3, 3, 1, 1, Ci)
        ws = torch.empty(max(conv.fd_ws_floats(*shp), 1), device=dev) if a.split else None
        for _ in range(5):
            conv.conv2d_fwd(x, wr, 1, 1, Cw=Ci, stats=stats, out=y, ws=ws)
        buf.zero_()
        torch.cuda.synchronize()
        nat.conv_halo_stamps(buf.data_ptr())
        conv.conv2d_fwd(x, wr, 1, 1, Cw=Ci, stats=stats, out=y, ws=ws)
        torch.cuda.synchronize()
        nat.conv_halo_stamps(0)
        s = buf.view(-1, 8).cpu()
        s = s[s[:, 1] != 0].double()
        pro, loop, epi = s[:, 2] - s[:, 1], s[:, 3] - s[:, 2], s[:, 4] - s[:, 3]
        rt = (s[:, 0] - s[:, 0].min()) * 10.0   # ns
        med = lambda t: float(t.median())
        print(json.dumps({"shape": key, "batch": a.batch, "wgs": int(s.shape[0]),
                          "prologue_cyc": med(pro), "loop_cyc": med(loop), "epilogue_cyc": med(epi),
                          "total_cyc": med(s[:, 4] - s[:, 1]),
                          "start_spread_us": round(float(rt.max()) / 1e3, 2),
                          "start_quartiles_us": [round(float(torch.quantile(rt, q)) / 1e3, 2) for q in (0.25, 0.5, 0.75)]}),
              flush=True)


if __name__ == "__main__":
    main()
