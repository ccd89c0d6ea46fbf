#!/bin/bash
# LeNet headline: bench wall clock vs rocprofv3 kernel trace of the SAME bench config (reconcile).
set -u
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 300 python bench.py --json-out $O/bench_plain.json > $O/bench_plain.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --json-out $O/bench_prof.json > $O/bench_prof.log 2>&1 || exit $?
T=$(ls $O/kt/*/run_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$T" ] || T=$(ls $O/kt/run_kernel_trace.csv)
python tools/reconcile_lenet.py $T $O/bench_prof.json $O/bench_plain.json > $O/reconcile.json 2>&1
cp $(dirname $T)/run_kernel_stats.csv $O/kernel_stats.csv
rm -f $T
echo done
