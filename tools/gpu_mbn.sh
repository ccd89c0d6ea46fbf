#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "depthwise or dgrad or fwd" > gpurun_out/mbn_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model mobilenet --steps 2 --warmup 1 > gpurun_out/bench_mobilenet.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mbn -o run --output-format csv -- python bench.py --model mobilenet --steps 1 --warmup 1 > gpurun_out/prof_mbn.log 2>&1 || exit $?
