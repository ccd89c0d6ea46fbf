#!/bin/bash
set -u
O=gpurun_out/r3f1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_native_mode_gpu.py -q -x --timeout 200 --timeout-method thread > $O/native_mode.log 2>&1; rc=$?
echo "native_mode rc=$rc $(tail -1 $O/native_mode.log)" >> $O/summary.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_r3_sysvar.sh
