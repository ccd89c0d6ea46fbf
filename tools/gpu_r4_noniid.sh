#!/bin/bash
# Round-4 non-IID (BASELINE config 3) death-rate sweep: ResNet-18, 2 label shards per client, reference
# round semantics (tools/fedavg_sim.py), native HIP engine vs fp32 PyTorch vs PyTorch autocast-bf16, 3 seeds,
# 2 and 8 clients at lr 0.1 (reference) and 8 clients at lr 0.02.  One JSONL per run under gpurun_out/$T.
T=${1:-r4n}
ROUNDS=${ROUNDS:-6}
mkdir -p gpurun_out/$T
args=()
for cl in ${CLIENTS:-2 8}; do
  for lr in ${LRS:-0.1}; do
    for eng in ${ENGINES:-native fp32 bf16}; do
      for s in ${SEEDS:-17 18 19}; do
        n="c${cl}_lr${lr}_${eng}_s${s}"
        args+=("$n" 300 "python tools/fedavg_sim.py --model resnet18 --clients $cl --noniid 2 --rounds $ROUNDS --engine $eng --lr $lr --seed $s --out gpurun_out/$T/$n.jsonl")
      done
    done
  done
done
bash tools/gpu_steps.sh $T "${args[@]}"
