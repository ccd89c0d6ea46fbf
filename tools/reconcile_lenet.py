"""Reconcile a rocprofv3 kernel trace of ``bench.py`` (LeNet) with the bench's own wall clock.

usage: python tools/reconcile_lenet.py <run_kernel_trace.csv> <bench.json under the profiler> [bench.json without]

Splits the trace into federated rounds (391 ``lenet_sample_step`` dispatches each, plus the eval and
SGD kernels between them), and for the LAST ``steps`` rounds (the timed ones) reports per round:
  span    first kernel start -> last kernel end of the round
  busy    union of kernel intervals (overlaps counted once)
  sum     plain sum of kernel durations
  gaps    span - busy (dispatch gaps between dependent graph nodes)
and the per-kernel median duration, next to the bench's ms_per_step with and without the profiler.
Per round, busy <= span <= wall must hold; if the profiled kernels are longer than the unprofiled
wall allows, the profiler itself is stretching them (it is: each traced dispatch carries a completion
signal and the packet processor serialises them).
"""
import csv
import json
import statistics
import sys


def _rows(path):
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            yield r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])


def _union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(argv):
    trace, prof_json = argv[0], argv[1]
    bench = json.loads(open(prof_json).read().strip().splitlines()[-1])
    plain = json.loads(open(argv[2]).read().strip().splitlines()[-1]) if len(argv) > 2 else None
    ks = sorted((s, e, n) for n, s, e in _rows(trace))
    step_name = "lenet_sample_step"
    # round boundaries: every 391st sample-step dispatch opens a round
    starts = [i for i, (s, e, n) in enumerate(ks) if step_name in n]
    per_round = 391
    first_of_round = starts[::per_round]
    rounds = []
    for j, i0 in enumerate(first_of_round):
        i1 = first_of_round[j + 1] if j + 1 < len(first_of_round) else len(ks)
        iv = [(s, e) for s, e, _ in ks[i0:i1]]
        span = max(e for _, e in iv) - min(s for s, _ in iv)
        busy = _union(iv)
        rounds.append({"span_ms": span / 1e6, "busy_ms": busy / 1e6, "sum_ms": sum(e - s for s, e in iv) / 1e6,
                       "gaps_ms": (span - busy) / 1e6, "kernels": i1 - i0})
    timed = rounds[-int(bench["steps"]):]
    med = {}
    for s, e, n in ks:
        key = n.split("(")[0]
        med.setdefault(key, []).append(e - s)
    out = {
        "rounds_in_trace": len(rounds),
        "timed_rounds": len(timed),
        "profiled_bench_ms_per_round": bench["ms_per_step"],
        "unprofiled_bench_ms_per_round": plain["ms_per_step"] if plain else None,
        "timed_round_span_ms_median": statistics.median(r["span_ms"] for r in timed),
        "timed_round_busy_ms_median": statistics.median(r["busy_ms"] for r in timed),
        "timed_round_kernel_sum_ms_median": statistics.median(r["sum_ms"] for r in timed),
        "timed_round_gaps_ms_median": statistics.median(r["gaps_ms"] for r in timed),
        "kernels_per_round": timed[-1]["kernels"],
        "kernel_median_us": {k: statistics.median(v) / 1e3 for k, v in med.items()},
        "kernel_calls": {k: len(v) for k, v in med.items()},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
