#!/bin/bash
# CNN-zoo kernels on the GPU box: numerics tests, ResNet engine tests, conv micro-bench.
set -u
mkdir -p gpurun_out
stop() { echo "STOP: step exited $1" >> gpurun_out/cnn_summary.txt; exit "$1"; }
timeout -k 10 300 python -m pytest tests/test_cnn_kernels_gpu.py -q -x > gpurun_out/cnn_tests.log 2>&1; rc=$?
echo "cnn tests rc=$rc" >> gpurun_out/cnn_summary.txt; tail -3 gpurun_out/cnn_tests.log >> gpurun_out/cnn_summary.txt
[ $rc -le 1 ] || stop $rc
timeout -k 10 400 python -m pytest tests/test_cnn_native_gpu.py -q -x > gpurun_out/resnet_tests.log 2>&1; rc=$?
echo "resnet tests rc=$rc" >> gpurun_out/cnn_summary.txt; tail -3 gpurun_out/resnet_tests.log >> gpurun_out/cnn_summary.txt
[ $rc -le 1 ] || stop $rc
timeout -k 10 240 python tools/bench_conv.py > gpurun_out/bench_conv.log 2>&1; rc=$?
echo "bench_conv rc=$rc" >> gpurun_out/cnn_summary.txt; tail -1 gpurun_out/bench_conv.log >> gpurun_out/cnn_summary.txt
[ $rc -eq 0 ] || stop $rc
echo done >> gpurun_out/cnn_summary.txt
