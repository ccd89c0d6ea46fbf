#!/bin/bash
# Round-4: grouped convs with narrow groups as one dense MFMA conv over a block-diagonal weight image.
T=${1:-r4g}
export TMPDIR=/tmp
O=gpurun_out/$T
bash tools/gpu_steps.sh $T \
  ntests 500 "python -u -m pytest tests/test_native_mode_gpu.py -x -q --timeout 240 --timeout-method thread" \
  prof_DPN26 300 "rocprofv3 --kernel-trace --stats -d $O/prof_DPN26 -o run --output-format csv -- python tools/prof_native_mode.py DPN26 13 && python tools/zoo_step_kernels.py \$(find $O/prof_DPN26 -name '*kernel_trace.csv' | head -1) 10 > $O/kernels_DPN26.txt && rm -rf $O/prof_DPN26" \
  bench 400 "BENCH_MODES=fp32,native-graph python tools/bench_hybrid.py DPN26 ResNeXt29_32x4d RegNetY_400MF RegNetX_200MF densenet_cifar > $O/bench_hybrid.jsonl"
