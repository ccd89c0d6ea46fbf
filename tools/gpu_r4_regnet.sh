#!/bin/bash
# RegNetY parity at lr 0.005 (and lr 0.02 for the record, allowed to fail), then the rest of the native-mode suite.
T=${1:-r4rg}
bash tools/gpu_steps.sh $T \
  reg 300 "python -u -m pytest 'tests/test_native_mode_gpu.py::test_family_trains_like_fp32' -q --timeout 240 --timeout-method thread -k RegNetY" \
  ntests 500 "python -u -m pytest tests/test_native_mode_gpu.py -q --timeout 240 --timeout-method thread"
