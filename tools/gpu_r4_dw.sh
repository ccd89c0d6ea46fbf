#!/bin/bash
# Round-4: depthwise stride-2 3x3 DGRAD fast path (CNN kernel + engine tests, MobileNet bench) and the
# LeNet backward stamps.
T=${1:-r4dw}
export TMPDIR=/tmp
bash tools/gpu_steps.sh $T \
  ctests 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread" \
  mbn 300 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/$T/mbn.json" \
  stamps 120 "env FEDMI_NATIVE_VARIANT=stamps python tools/diag_stamps.py > gpurun_out/$T/stamps.log 2>&1"
