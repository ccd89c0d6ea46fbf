#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests/test_cnn_native_gpu.py -q > gpurun_out/resnet_tests.log 2>&1; rc=$?
echo "engine tests rc=$rc" > gpurun_out/cnn3_summary.txt; tail -6 gpurun_out/resnet_tests.log >> gpurun_out/cnn3_summary.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python tools/diag_cnn_train.py ResNet18 0.1 3 > gpurun_out/diag_train.log 2>&1; rc=$?
echo "diag rc=$rc" >> gpurun_out/cnn3_summary.txt; cat gpurun_out/diag_train.log | grep -v amdgpu >> gpurun_out/cnn3_summary.txt
