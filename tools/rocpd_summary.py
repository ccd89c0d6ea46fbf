"""Per-kernel totals from a rocprofv3 rocpd database (``-o run`` -> run_results.db), CSV-like text.

    python tools/rocpd_summary.py gpurun_out/x/run_results.db [top]
"""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = list(c.execute(f"select {name}, count(*), sum(end - start) from kernels group by {name} order by 3 desc"))
tot = sum(r[2] for r in rows)
print(f"# total GPU kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches")
print("name,calls,total_ms,avg_us,pct")
for n, k, t in rows[:top]:
    print(f"{n[:90]},{k},{t / 1e6:.3f},{t / k / 1e3:.2f},{100 * t / tot:.1f}")
