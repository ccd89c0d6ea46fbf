#!/bin/bash
# Round-4: LeNet KS2 phase stamps + a kernel trace of the headline bench (summary only).
T=${1:-r4s5}
export TMPDIR=/tmp
bash tools/gpu_steps.sh $T \
  stamps 120 "FEDMI_NATIVE_VARIANT=stamps python tools/diag_stamps.py" \
  prof 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o p --output-format csv -- python bench.py --steps 5 --warmup 2 --json-out gpurun_out/$T/bench_prof.json"
python tools/trace_top.py gpurun_out/$T/prof/p_kernel_trace.csv > gpurun_out/$T/lenet_top.txt 2>&1
rm -f gpurun_out/$T/prof/p_kernel_trace.csv
exit 0
