#!/bin/bash
# Round-4: off-grid depthwise convs on padded channels (PNASNetA): native-mode tests, bench.
T=${1:-r4p}
bash tools/gpu_steps.sh $T \
  ntests 500 "python -u -m pytest tests/test_native_mode_gpu.py -x -q --timeout 240 --timeout-method thread" \
  bench 300 "BENCH_MODES=fp32,native-graph python tools/bench_hybrid.py PNASNetA PNASNetB ShuffleNetV2 > gpurun_out/$T/bench_hybrid.jsonl"
