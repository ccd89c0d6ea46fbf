#!/bin/bash
# Round-4: conv_tap with the conflict-free LDS swizzle ((r >> 1) & 7): kernel tests, per-shape timings,
# one PMC pass on the l2 forward, ResNet-18 / MobileNet bench steps.
T=${1:-r4c}
export TMPDIR=/tmp
bash tools/gpu_steps.sh $T \
  ctests 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 200 --timeout-method thread" \
  taps 200 "python tools/bench_tap.py --graph --iters 50 > gpurun_out/$T/conv_shapes.jsonl" \
  pmc 60 "rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY -d gpurun_out/$T/pmc -o p --output-format csv -- python tools/bench_tap.py --shapes l2 --passes fwd_nostats --iters 20" \
  r18 300 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/$T/r18.json" \
  mbn 300 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/$T/mbn.json"
