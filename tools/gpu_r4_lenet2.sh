#!/bin/bash
# Round-4: LeNet tests after the conv1-bias fix, the N=8 projection with the polling checkpoint writer,
# and an A/B with the Python writer (FEDMI_NATIVE_CKPT=0).
T=${1:-r4l2}
bash tools/gpu_steps.sh $T \
  tests 600 "python -u -m pytest tests/test_lenet_kernels_gpu.py tests/test_kernel_list_gpu.py tests/test_eval_ckpt.py tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py tests/test_native_mode_gpu.py tests/test_hybrid_graph_gpu.py tests/test_flat_ops_gpu.py -v --timeout 200 --timeout-method thread" \
  asan 120 "ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0 ./tools/asan/bin/lenet_engine_asan" \
  proj8 120 "python bench.py --breakdown --project-world 8 --steps 40 --warmup 5 --json-out gpurun_out/$T/proj8.json" \
  proj8py 120 "FEDMI_NATIVE_CKPT=0 python bench.py --breakdown --project-world 8 --steps 40 --warmup 5 --json-out gpurun_out/$T/proj8py.json" \
  bench 120 "python bench.py --json-out gpurun_out/$T/bench1.json"
