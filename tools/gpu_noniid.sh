#!/bin/bash
# BASELINE config 3 at its stated scale: ResNet-18 FedAvg over 8 clients x 2 label shards, 20 rounds (the reference's
# round count, src/server.py:120), native vs deterministic fp32 PyTorch vs deterministic PyTorch autocast-bf16,
# seeds 1-3, one learning rate per call (tools/fedavg_sim.py, all clients in one process on one GPU).
#   usage: bash tools/gpu_noniid.sh <tag> <lr> [rounds] [clients] [engines]
T=${1:-r5_noniid}; LR=${2:-0.02}; ROUNDS=${3:-20}; CL=${4:-8}; ENG=${5:-"native fp32 bf16"}
args=()
for e in $ENG; do
  args+=("${e}_lr$LR" 900 "python -u tools/fedavg_sim.py --model resnet18 --clients $CL --noniid 2 --rounds $ROUNDS --lr $LR --engine $e --seeds 1,2,3 --deterministic --out gpurun_out/$T/c${CL}_${e}_lr$LR.jsonl")
done
bash tools/gpu_steps.sh "$T" "${args[@]}"
