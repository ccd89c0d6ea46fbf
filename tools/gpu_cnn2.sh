#!/bin/bash
# Native CNN engine tests + ResNet-18 / MobileNet FedAvg benches on one GPU.
set -u
mkdir -p gpurun_out
stop() { echo "STOP: step exited $1" >> gpurun_out/cnn2_summary.txt; exit "$1"; }
timeout -k 10 700 python -m pytest tests/test_cnn_native_gpu.py -q > gpurun_out/resnet_tests.log 2>&1; rc=$?
echo "engine tests rc=$rc" >> gpurun_out/cnn2_summary.txt; tail -4 gpurun_out/resnet_tests.log >> gpurun_out/cnn2_summary.txt
[ $rc -le 1 ] || stop $rc
timeout -k 10 400 python bench.py --model resnet18 --noniid 2 --steps 2 --warmup 1 > gpurun_out/bench_r18.log 2>&1; rc=$?
echo "bench resnet18 rc=$rc" >> gpurun_out/cnn2_summary.txt; tail -2 gpurun_out/bench_r18.log >> gpurun_out/cnn2_summary.txt
[ $rc -eq 0 ] || stop $rc
timeout -k 10 400 python bench.py --model mobilenet --steps 2 --warmup 1 > gpurun_out/bench_mb.log 2>&1; rc=$?
echo "bench mobilenet rc=$rc" >> gpurun_out/cnn2_summary.txt; tail -2 gpurun_out/bench_mb.log >> gpurun_out/cnn2_summary.txt
[ $rc -eq 0 ] || stop $rc
echo done >> gpurun_out/cnn2_summary.txt
