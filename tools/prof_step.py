#!/usr/bin/env python
"""Per-dispatch timeline of ONE training step from a rocprofv3 kernel trace
(the step starting at the k-th occurrence of a marker kernel).

    python tools/prof_step.py gpurun_out/prof_r18/run_kernel_trace.csv [k] [marker]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    marker = sys.argv[3] if len(sys.argv) > 3 else "sched_next"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[k], idx[k + 1]
    busy = 0.0
    for r in rows[a:b]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy += d
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        n = n.split("(")[0][-34:]
        wg = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{d:8.2f} us  wgs={wg:6d} z={r['Grid_Size_Z']:>3s} lds={r['LDS_Block_Size']:>6s} vgpr={r['VGPR_Count']:>4s}  {n}")
    span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
    print(f"busy {busy:.1f} us, span {span:.1f} us, {b - a} dispatches")


if __name__ == "__main__":
    main()
