#!/bin/bash
# GoogLeNet native engine on the GPU: the new kernels (maxpool3, strided BN, dgrad accumulate), the engine
# tests, then native vs PyTorch-layer bench lines.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "maxpool3 or strided or accumulate" > gpurun_out/goog_kernels.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_cnn_native_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k GoogLeNet > gpurun_out/goog_engine.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model googlenet --steps 2 --warmup 1 > gpurun_out/bench_googlenet.log 2>&1 || exit $?
FEDMI_TORCH_PATH=1 timeout -k 10 300 python bench.py --model googlenet --steps 2 --warmup 1 \
  > gpurun_out/bench_googlenet_torchpath.log 2>&1 || exit $?
