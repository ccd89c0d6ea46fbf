#!/bin/bash
# Round-4 batch 4: conv_tap split-K combined in-kernel by the last-arriving split (no combine launch);
# LeNet KS2 with unconditional parameter loads in the FC weight tiles.
T=${1:-r4b4}
bash tools/gpu_steps.sh $T \
  ctests 400 "python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py -q --timeout 200 --timeout-method thread" \
  ltests 200 "python -u -m pytest tests/test_lenet_kernels_gpu.py -q --timeout 120 --timeout-method thread" \
  taps 120 "python tools/bench_tap.py --graph --iters 50 --passes fwd_stats,fwd_nostats,dgrad_tap > gpurun_out/$T/conv_shapes.jsonl" \
  stamps 120 "FEDMI_NATIVE_VARIANT=stamps python tools/diag_stamps.py" \
  bench 120 "python bench.py --json-out gpurun_out/$T/bench1.json" \
  r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/$T/r18.json" \
  mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/$T/mbn.json"
