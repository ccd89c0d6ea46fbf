#!/bin/bash
# Round-4 validation: the whole GPU suite, LeNet stamps (with KS2 roles), ResNet-18 / MobileNet bench rounds.
T=${1:-r4f}
bash tools/gpu_steps.sh $T \
  gpusuite 900 "python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  stamps 120 "FEDMI_NATIVE_VARIANT=stamps python tools/diag_stamps.py" \
  bench 120 "python bench.py --json-out gpurun_out/$T/bench1.json" \
  r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/$T/r18.json" \
  mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/$T/mbn.json"
