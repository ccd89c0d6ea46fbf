#!/bin/bash
# Round-4 diagnostics: checkpoint I/O probe, per-tensor gradient cosines (native vs emulated vs fp32 vs
# torch-bf16), the non-IID lr-0.1 bisect (native / fp32 / torch-bf16 stepped on identical batches), and the
# GPU tests touched by the fixed-order CE loss sums.
T=${1:-r4d}
mkdir -p gpurun_out/$T
bash tools/gpu_steps.sh $T \
  ckio 120 "python tools/probe_ckpt_io.py" \
  tests 400 "python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_lenet_kernels_gpu.py tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -k 'head or eval or determin or graph or match'" \
  cos 300 "python tools/diag_grad_cosines.py --models ResNet18 MobileNetV2 --out gpurun_out/$T/grad_cosines.jsonl" \
  bisect 500 "python tools/diag_noniid_bisect.py --steps 150 --out gpurun_out/$T/bisect_s17.jsonl"
