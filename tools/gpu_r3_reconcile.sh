#!/bin/bash
# LeNet bench.py under rocprofv3 vs without: per-round kernel span / busy / sum against the bench wall clock
set -u
O=gpurun_out/r3rec
mkdir -p $O
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --json-out $O/bench_noprof.json > $O/bench_noprof.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 5 --warmup 2 --json-out $O/bench_prof.json > $O/bench_prof.log 2>&1 || exit $?
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
S=$(find $O/prof -name "run_kernel_stats.csv" | head -1)
python tools/reconcile_lenet.py "$T" $O/bench_prof.json $O/bench_noprof.json > $O/reconcile.txt 2>&1; rc=$?
cp "$S" $O/kernel_stats.csv
rm -f "$T"
exit $rc
