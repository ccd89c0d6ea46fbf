#!/bin/bash
# Round-4 zoo backend: concat buffers, BN-counter fold, O-padded / batched packs, row-strided unpads,
# BN-backward + gradient-accumulation fusion.  native-mode GPU tests, per-step kernels, fp32 vs native-graph.
#   usage: bash tools/gpu_r4_zoo.sh <tag> [prof models...]
T=${1:-r4z}; shift
PROF=${*:-densenet_cifar RegNetY_400MF}
export TMPDIR=/tmp
O=gpurun_out/$T
args=(ntests 500 "python -u -m pytest tests/test_native_mode_gpu.py -x -q --timeout 240 --timeout-method thread")
for m in $PROF; do
  args+=(prof_$m 300 "rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python tools/prof_native_mode.py $m 13 && python tools/zoo_step_kernels.py \$(find $O/prof_$m -name '*kernel_trace.csv' | head -1) 10 > $O/kernels_$m.txt && rm -rf $O/prof_$m")
done
args+=(bench 560 "BENCH_MODES=fp32,native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 RegNetY_400MF ShuffleNetG2 DPN26 > $O/bench_hybrid.jsonl")
bash tools/gpu_steps.sh $T "${args[@]}"
