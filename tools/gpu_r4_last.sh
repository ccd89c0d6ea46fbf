#!/bin/bash
# Round-4 last box check: the whole GPU suite, smoke(), the headline bench at defaults, ResNet-18 / MobileNet.
T=${1:-r4last}
bash tools/gpu_steps.sh $T \
  gpusuite 900 "python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  smoke 180 "python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  bench 150 "python bench.py --json-out gpurun_out/$T/bench1.json" \
  r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/$T/r18.json" \
  mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/$T/mbn.json"
