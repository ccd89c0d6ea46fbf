#!/bin/bash
# ResNet-18 kernel tests + engine tests + bench + kernel profile (one GPU box session).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r18_tests.log 2>&1; rc=$?
echo "tests rc=$rc" > gpurun_out/r18_summary.txt; tail -15 gpurun_out/r18_tests.log >> gpurun_out/r18_summary.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model resnet18 --steps 2 --warmup 1 > gpurun_out/bench_resnet18.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r18 -o run --output-format csv -- python bench.py --model resnet18 --steps 1 --warmup 1 > gpurun_out/prof_r18.log 2>&1 || exit $?
echo done >> gpurun_out/r18_summary.txt
timeout -k 10 120 python tools/bench_tap.py --iters 30 > gpurun_out/bench_tap.log 2>&1 || exit $?
