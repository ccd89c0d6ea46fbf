#!/bin/bash
# Row-reduction microbenchmark (two-launch vs last-arriver finalize) at zoo BN shapes, with a kernel trace.
T=${1:-r4rows}
export TMPDIR=/tmp
O=gpurun_out/$T
SH="131072:48 131072:64 131072:256 32768:512 8192:384 8192:1024 2048:1024 2048:2432"
bash tools/gpu_steps.sh $T \
  rows 120 "python tools/bench_rows.py $SH > $O/rows.jsonl" \
  rows_prof 180 "rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/bench_rows.py $SH && python tools/trace_top.py \$(find $O/prof -name '*kernel_trace.csv' | head -1) > $O/rows_top.txt; rm -rf $O/prof"
