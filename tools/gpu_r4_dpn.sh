#!/bin/bash
# Round-4: DPN's paired slice gradients summed as two copies: native-mode tests, DPN26 kernels, bench.
T=${1:-r4d}
export TMPDIR=/tmp
O=gpurun_out/$T
bash tools/gpu_steps.sh $T \
  ntests 500 "python -u -m pytest tests/test_native_mode_gpu.py -x -q --timeout 240 --timeout-method thread" \
  prof_DPN26 300 "rocprofv3 --kernel-trace --stats -d $O/prof_DPN26 -o run --output-format csv -- python tools/prof_native_mode.py DPN26 13 && python tools/zoo_step_kernels.py \$(find $O/prof_DPN26 -name '*kernel_trace.csv' | head -1) 10 > $O/kernels_DPN26.txt && rm -rf $O/prof_DPN26" \
  bench 300 "BENCH_MODES=fp32,native-graph python tools/bench_hybrid.py DPN26 DPN92 > $O/bench_hybrid.jsonl"
