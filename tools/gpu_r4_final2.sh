#!/bin/bash
# Round-4 final validation, part 2: smoke(), the headline bench at defaults, ResNet-18 / MobileNet rounds, zoo bench.
T=${1:-r4v2}
bash tools/gpu_steps.sh $T \
  smoke 180 "python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  bench 150 "python bench.py --json-out gpurun_out/$T/bench1.json" \
  r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/$T/r18.json" \
  mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/$T/mbn.json" \
  zoo 300 "BENCH_MODES=fp32,native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 RegNetY_400MF DPN26 SENet18 EfficientNetB0 > gpurun_out/$T/zoo.jsonl"
