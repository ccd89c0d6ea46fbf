#!/bin/bash
# Round-4: LeNet KS1 with W1 register-resident for fc1 forward + dX (no transposed fc1 image): kernel tests,
# bench, per-phase stamps; then the N=8 projection under a kernel + memory-copy trace (checkpoint outliers).
T=${1:-r4l3}
bash tools/gpu_steps.sh $T \
  tests 300 "python -u -m pytest tests/test_lenet_kernels_gpu.py tests/test_kernel_list_gpu.py tests/test_eval_ckpt.py -v --timeout 200 --timeout-method thread" \
  bench 120 "python bench.py --json-out gpurun_out/$T/bench1.json" \
  stamps 200 "FEDMI_NATIVE_VARIANT=stamps python tools/diag_stamps.py"
[ -z "${PROF8:-}" ] || bash tools/gpu_steps.sh $T \
  prof8 240 "rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/$T/prof8 -o p --output-format csv -- python bench.py --breakdown --project-world 8 --steps 40 --warmup 5 --json-out gpurun_out/$T/proj8_prof.json"
