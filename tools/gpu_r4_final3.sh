#!/bin/bash
# Round-4 final validation after the O-limited WGRAD reduction: native-mode + CNN kernel tests, smoke(),
# the headline bench, ResNet-18 / MobileNet rounds, zoo bench.
T=${1:-r4v3}
bash tools/gpu_steps.sh $T \
  ntests 400 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_cnn_kernels_gpu.py -x -q --timeout 240 --timeout-method thread" \
  smoke 180 "python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  bench 150 "python bench.py --json-out gpurun_out/$T/bench1.json" \
  r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/$T/r18.json" \
  mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/$T/mbn.json" \
  zoo 300 "BENCH_MODES=fp32,native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 RegNetY_400MF DPN26 SENet18 EfficientNetB0 > gpurun_out/$T/zoo.jsonl"
