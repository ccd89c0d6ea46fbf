#!/usr/bin/env python
"""Summarise a rocprofv3 kernel-trace CSV: per kernel name the total / mean time and call count, plus the
busy time and wall span of the whole trace.  Used on the GPU box so only the summary travels back.

    python tools/trace_top.py <p_kernel_trace.csv> [--top 40]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    tot = collections.Counter()
    calls = collections.Counter()
    t0, t1, busy = None, None, 0
    for r in csv.DictReader(open(a.trace)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"]
        tot[name] += e - s
        calls[name] += 1
        busy += e - s
        t0 = s if t0 is None else min(t0, s)
        t1 = e if t1 is None else max(t1, e)
    if t0 is None:
        print("empty trace")
        return
    print(f"kernels {sum(calls.values())}  busy {busy / 1e6:.3f} ms  span {(t1 - t0) / 1e6:.3f} ms")
    for name, ns in tot.most_common(a.top):
        print(f"{ns / 1e3:11.1f} us {calls[name]:7d} calls {ns / calls[name] / 1e3:9.2f} us/call "
              f"{100.0 * ns / busy:5.1f}%  {name[:110]}")


if __name__ == "__main__":
    main()
