#!/bin/bash
# Round-4 non-IID root cause: the native engine dies in round 1 of the 2-client lr-0.1 split in the
# simulator (graph replay + augmentation) but trains in the eager no-augment bisect. One round each,
# native with augmentation / graph replay toggled, plus fp32 and torch-bf16 at the default.
T=${1:-r4na}
S=${SEED:-17}
R=${ROUNDS:-2}
base="python tools/fedavg_sim.py --model resnet18 --clients 2 --noniid 2 --rounds $R --lr 0.1 --seed $S"
bash tools/gpu_steps.sh $T \
  nat 240 "$base --engine native --out gpurun_out/$T/nat.jsonl" \
  nat_noaug 240 "$base --engine native --no-augment --out gpurun_out/$T/nat_noaug.jsonl" \
  nat_nograph 240 "$base --engine native --no-graph --out gpurun_out/$T/nat_nograph.jsonl" \
  nat_noaug_nograph 240 "$base --engine native --no-augment --no-graph --out gpurun_out/$T/nat_noaug_nograph.jsonl" \
  bf16 300 "$base --engine bf16 --out gpurun_out/$T/bf16.jsonl" \
  fp32 300 "$base --engine fp32 --no-augment --out gpurun_out/$T/fp32_noaug.jsonl"
