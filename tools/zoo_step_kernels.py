#!/usr/bin/env python
"""Per-step kernel breakdown of the LAST n graph-replayed zoo steps in a rocprofv3 kernel trace
(tools/prof_native_mode.py runs): kernels grouped by name, per-step time / count, and the step total.

    python tools/zoo_step_kernels.py <run_kernel_trace.csv> [n_steps]
"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
# steps: the fused SGD launch closes each step
sgd = [i for i, r in enumerate(rows) if "sgd" in r["Kernel_Name"].lower()]
if len(sgd) < n + 1:
    print(f"only {len(sgd)} SGD launches found")
    sys.exit(0)
a, b = sgd[-n - 1] + 1, sgd[-1] + 1
fam_t, fam_n = defaultdict(float), defaultdict(int)
busy = 0.0
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    k = k.split("(")[0][:70] or r["Kernel_Name"][:70]
    fam_t[k] += d
    fam_n[k] += 1
    busy += d
span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"steps {n}: busy {busy / n:.1f} us/step, span {span / n:.1f} us/step, {(b - a) / n:.0f} dispatches/step")
for k, t in sorted(fam_t.items(), key=lambda kv: -kv[1]):
    print(f"{t / n:9.1f} us  {fam_n[k] / n:6.1f}/step  {t / fam_n[k]:7.2f} us avg  {k}")
