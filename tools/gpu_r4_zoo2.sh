#!/bin/bash
# Round-4 zoo: native-mode GPU tests, per-step kernels, then fp32 / HEAD-baseline (base_head/) / current
# native-graph on one box.
T=${1:-r4z3}
export TMPDIR=/tmp
O=gpurun_out/$T
B=$PWD/$O
args=(ntests 500 "python -u -m pytest tests/test_native_mode_gpu.py -x -q --timeout 240 --timeout-method thread")
for m in densenet_cifar RegNetY_400MF DPN26; do
  args+=(prof_$m 300 "rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python tools/prof_native_mode.py $m 13 && python tools/zoo_step_kernels.py \$(find $O/prof_$m -name '*kernel_trace.csv' | head -1) 10 > $O/kernels_$m.txt && rm -rf $O/prof_$m")
done
args+=(base_dpn 300 "cd base_head && rocprofv3 --kernel-trace --stats -d $B/prof_base -o run --output-format csv -- python tools/prof_native_mode.py DPN26 13 && python tools/zoo_step_kernels.py \$(find $B/prof_base -name '*kernel_trace.csv' | head -1) 10 > $B/kernels_DPN26_base.txt && rm -rf $B/prof_base")
args+=(bench_base 400 "cd base_head && BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 RegNetY_400MF DPN26 > $B/bench_base.jsonl")
args+=(bench 560 "BENCH_MODES=fp32,native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 RegNetY_400MF ShuffleNetG2 DPN26 > $O/bench_hybrid.jsonl")
bash tools/gpu_steps.sh $T "${args[@]}"
