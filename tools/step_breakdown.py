#!/usr/bin/env python
"""Per-step kernel-time breakdown of a native CNN engine from a rocprofv3 kernel trace.

Steps are delimited by the engine's ``sched_next`` kernel; over steps [k0, k0 + n) it reports
the mean busy time per step (sum of kernel durations), the wall span per step, and the share of
each kernel family (BatchNorm apply / backward, conv forward / dgrad, weight gradient, depthwise,
head, SGD + weight repack, other).

    python tools/step_breakdown.py <run_kernel_trace.csv> [k0] [n] [--json out.json]
"""
import csv
import json
import sys
from collections import defaultdict

FAMILIES = [
    ("bn_fwd", ("bn_apply", "bn_coeff")),
    ("bn_bwd", ("bn_bwd",)),
    ("depthwise", ("dw_",)),
    ("wgrad", ("wgrad", "conv_igemm<2")),
    ("conv_fwd_dgrad", ("conv_tap", "conv_igemm<0", "conv_igemm<1", "conv_halo", "splitk_reduce", "dgrad_pack")),
    ("head", ("head_",)),
    ("sgd_pack", ("sgd_flat", "conv_pack", "pack_multi")),
    ("pool", ("maxpool",)),
]


def family(name: str) -> str:
    for fam, keys in FAMILIES:
        if any(k in name for k in keys):
            return fam
    return "other"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    path = args[0]
    k0 = int(args[1]) if len(args) > 1 else 20
    n = int(args[2]) if len(args) > 2 else 20
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "sched_next" in r["Kernel_Name"]]
    n = min(n, len(idx) - k0 - 1)
    fam_t = defaultdict(float)
    busy = span = 0.0
    disp = 0
    for s in range(k0, k0 + n):
        a, b = idx[s], idx[s + 1]
        span += (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
        for r in rows[a:b]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            busy += d
            fam_t[family(r["Kernel_Name"])] += d
            disp += 1
    res = {"trace": path, "steps": n, "busy_us_per_step": round(busy / n, 1), "span_us_per_step": round(span / n, 1),
           "dispatches_per_step": round(disp / n, 1),
           "share_pct": {f: round(100 * t / busy, 1) for f, t in sorted(fam_t.items(), key=lambda x: -x[1])},
           "us_per_step": {f: round(t / n, 1) for f, t in sorted(fam_t.items(), key=lambda x: -x[1])}}
    print(json.dumps(res, indent=1))
    if out:
        open(out, "w").write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
