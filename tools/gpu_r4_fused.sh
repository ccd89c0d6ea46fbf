#!/bin/bash
# Round-4: LeNet epoch as one fused launch per step (SGD of the previous step + grid barrier + samples).
T=${1:-r4fu}
bash tools/gpu_steps.sh $T \
  ltests 240 "python -u -m pytest tests/test_lenet_kernels_gpu.py tests/test_kernel_list_gpu.py -v --timeout 120 --timeout-method thread" \
  asan 120 "ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0 ./tools/asan/bin/lenet_engine_asan" \
  bench 120 "python bench.py --json-out gpurun_out/$T/bench1.json" \
  bench2 120 "python bench.py --json-out gpurun_out/$T/bench2.json" \
  proj8 120 "python bench.py --breakdown --project-world 8 --steps 40 --warmup 5 --json-out gpurun_out/$T/proj8.json"
