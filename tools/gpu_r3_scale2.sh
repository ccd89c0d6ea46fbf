#!/bin/bash
# 8-rank rehearsal + peer/RCCL tests at HEAD, then a rocprofv3 kernel breakdown of the -c Y kernels
set -u
STAGES="tests reh8" bash tools/gpu_r3_scale.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/r3ck
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ck/prof -o run -- python tools/bench_compress.py > gpurun_out/r3ck/bench.log 2>&1; rc=$?
echo "compress prof rc=$rc" >> gpurun_out/r3s/summary.txt
find gpurun_out/r3ck/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r3ck/kernel_stats.csv \;
find gpurun_out/r3ck/prof -name "*kernel_trace.csv" -size +20M -delete
exit $rc
