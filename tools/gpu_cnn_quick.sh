#!/bin/bash
# CNN kernel + engine GPU tests, then ResNet-18 / MobileNet / VGG16 / PreActResNet18 bench lines.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/cnn_tests.log 2>&1 || exit $?
for m in resnet18 mobilenet vgg16 preactresnet18; do
  timeout -k 10 300 python bench.py --model $m --steps 2 --warmup 1 > gpurun_out/bench_$m.log 2>&1 || exit $?
done
