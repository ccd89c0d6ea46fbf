#!/bin/bash
# Round-4 batch 2: LeNet kernel tests (no-augment case fixed), conv_tap 3- vs 4-stage A/B interleaved in
# one box (tap3 build variant), non-IID lr-0.1 death rates over seeds (2 clients x 1 round, 10 seeds;
# 8 clients x 3 rounds, 3 seeds) for native / torch-bf16 / fp32.
T=${1:-r4b2}
S10=1,2,3,4,5,6,7,8,9,10
base2="python tools/fedavg_sim.py --model resnet18 --clients 2 --noniid 2 --rounds 1 --lr 0.1 --seeds $S10"
base8="python tools/fedavg_sim.py --model resnet18 --clients 8 --noniid 2 --rounds 3 --lr 0.1 --seeds 1,2,3"
tap="python tools/bench_tap.py --graph --iters 50 --shapes l1,l2,l3,l4,d2,d4 --passes fwd_nostats,dgrad_tap"
bash tools/gpu_steps.sh $T \
  ltests 200 "python -u -m pytest tests/test_lenet_kernels_gpu.py -q --timeout 120 --timeout-method thread" \
  tapA1 60 "$tap > gpurun_out/$T/tap4_1.jsonl" \
  tapB1 60 "FEDMI_NATIVE_VARIANT=tap3 $tap > gpurun_out/$T/tap3_1.jsonl" \
  tapA2 60 "$tap > gpurun_out/$T/tap4_2.jsonl" \
  tapB2 60 "FEDMI_NATIVE_VARIANT=tap3 $tap > gpurun_out/$T/tap3_2.jsonl" \
  tapA3 60 "$tap > gpurun_out/$T/tap4_3.jsonl" \
  tapB3 60 "FEDMI_NATIVE_VARIANT=tap3 $tap > gpurun_out/$T/tap3_3.jsonl" \
  d2nat 200 "$base2 --engine native --out gpurun_out/$T/c2_native.jsonl" \
  d2bf16 300 "$base2 --engine bf16 --out gpurun_out/$T/c2_bf16.jsonl" \
  d2fp32 300 "$base2 --engine fp32 --out gpurun_out/$T/c2_fp32.jsonl" \
  d8nat 200 "$base8 --engine native --out gpurun_out/$T/c8_native.jsonl" \
  d8bf16 300 "$base8 --engine bf16 --out gpurun_out/$T/c8_bf16.jsonl" \
  d8fp32 300 "$base8 --engine fp32 --out gpurun_out/$T/c8_fp32.jsonl"
