#!/bin/bash
# Round-4 batch 3: conv_tap 3- vs 4-stage A/B (interleaved, one box), the checkpoint-writer experiment at
# the N=8 projection cadence, then the non-IID lr-0.1 death-rate sweep over 6 rounds x 10 seeds.
T=${1:-r4b3}
tap="python tools/bench_tap.py --graph --iters 50 --shapes l1,l2,l3,l4,d2,d4 --passes fwd_nostats,dgrad_tap"
bash tools/gpu_steps.sh $T \
  tapA1 60 "$tap > gpurun_out/$T/tap4_1.jsonl" \
  tapB1 60 "FEDMI_NATIVE_VARIANT=tap3 $tap > gpurun_out/$T/tap3_1.jsonl" \
  tapA2 60 "$tap > gpurun_out/$T/tap4_2.jsonl" \
  tapB2 60 "FEDMI_NATIVE_VARIANT=tap3 $tap > gpurun_out/$T/tap3_2.jsonl" \
  tapA3 60 "$tap > gpurun_out/$T/tap4_3.jsonl" \
  tapB3 60 "FEDMI_NATIVE_VARIANT=tap3 $tap > gpurun_out/$T/tap3_3.jsonl" && \
bash tools/gpu_r4_ckpt.sh r4k && \
bash tools/gpu_steps.sh $T \
  s6nat 200 "python tools/fedavg_sim.py --model resnet18 --clients 2 --noniid 2 --rounds 6 --lr 0.1 --seeds 1,2,3,4,5,6,7,8,9,10 --engine native --out gpurun_out/$T/r6_native.jsonl" \
  s6bf16 400 "python tools/fedavg_sim.py --model resnet18 --clients 2 --noniid 2 --rounds 6 --lr 0.1 --seeds 1,2,3,4,5,6,7,8,9,10 --engine bf16 --out gpurun_out/$T/r6_bf16.jsonl" \
  s6fp32 500 "python tools/fedavg_sim.py --model resnet18 --clients 2 --noniid 2 --rounds 6 --lr 0.1 --seeds 1,2,3,4,5,6,7,8,9,10 --engine fp32 --out gpurun_out/$T/r6_fp32.jsonl"
