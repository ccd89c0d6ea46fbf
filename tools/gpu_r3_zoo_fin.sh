#!/bin/bash
# zoo backend after the one-pass BN finalize: native-mode GPU tests, then per-step kernels + bench
set -u
mkdir -p gpurun_out/r3zf
timeout -k 10 500 python -u -m pytest tests/test_native_mode_gpu.py -q -x --timeout 240 --timeout-method thread > gpurun_out/r3zf/tests.log 2>&1; rc=$?
echo "native_mode tests rc=$rc $(tail -1 gpurun_out/r3zf/tests.log)" > gpurun_out/r3zf/summary.txt
if [ $rc -ne 0 ]; then exit $rc; fi
STAGES="prof bench" bash tools/gpu_r3_zoo_prof.sh
