#!/bin/bash
# Round-4: LeNet backward shifted-copy builds as 16-byte row segments: kernel tests, stamps, headline bench x2.
T=${1:-r4l4}
export TMPDIR=/tmp
bash tools/gpu_steps.sh $T \
  ltests 300 "python -u -m pytest tests/test_lenet_kernels_gpu.py -x -q --timeout 200 --timeout-method thread" \
  stamps 120 "env FEDMI_NATIVE_VARIANT=stamps python tools/diag_stamps.py > gpurun_out/$T/stamps.log 2>&1" \
  bench_a 150 "python bench.py --json-out gpurun_out/$T/bench_a.json" \
  bench_b 150 "python bench.py --json-out gpurun_out/$T/bench_b.json"
