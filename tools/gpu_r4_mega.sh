#!/bin/bash
# Round-4 batch: LeNet (fc1 W1-in-registers, fc3 in LDS) tests/bench/stamps, conv_tap 4-stage tests and
# timings, CNN kernel profiles, non-IID lr-0.1 A/B.  Each part stops the chain on a crash-class exit.
bash tools/gpu_r4_lenet3.sh r4l4 && \
bash tools/gpu_steps.sh r4c2 \
  ctests 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread" \
  taps 200 "python tools/bench_tap.py --graph --iters 50 > gpurun_out/r4c2/conv_shapes.jsonl" && \
bash tools/gpu_r4_cnnprof.sh r4cp && \
bash tools/gpu_r4_noniid_ab.sh r4na
