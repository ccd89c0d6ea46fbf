#!/bin/bash
# Round-4 closing confirmation: native-mode suite, smoke(), one zoo bench row.
T=${1:-r4c9}
bash tools/gpu_steps.sh $T \
  ntests 500 "python -u -m pytest tests/test_native_mode_gpu.py -q --timeout 240 --timeout-method thread" \
  smoke 180 "python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  zoo 300 "BENCH_MODES=fp32,native-graph python tools/bench_hybrid.py densenet_cifar RegNetY_400MF > gpurun_out/$T/zoo.jsonl"
