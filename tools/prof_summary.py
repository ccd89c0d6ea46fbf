#!/usr/bin/env python
"""Summarise a rocprofv3 kernel-stats CSV: per-kernel total/avg time and the
per-training-step share (steps counted by a marker kernel).

    python tools/prof_summary.py gpurun_out/prof_r18/run_kernel_stats.csv [marker] [top]
"""
import csv
import sys


def short(name: str) -> str:
    if "conv_igemm" in name:
        return name[name.find("conv_igemm"):].split("(")[0]
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][-60:]


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "sched_next"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    steps = sum(int(r["Calls"]) for r in rows if marker in r["Name"]) or 1
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    agg = {}
    for r in rows:
        k = short(r["Name"])
        a = agg.setdefault(k, [0.0, 0])
        a[0] += float(r["TotalDurationNs"])
        a[1] += int(r["Calls"])
    print(f"total {tot / 1e6:.2f} ms over {steps} steps -> {tot / 1e3 / steps:.1f} us/step")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t / 1e3 / steps:9.1f} us/step {c / steps:6.1f} calls/step {t / c / 1e3:8.2f} us/call {100 * t / tot:5.1f}%  {k}")


if __name__ == "__main__":
    main()
