#!/bin/bash
# -c Y accuracy sweep at 8 ranks on one GPU (bench.py --gpus 8 rehearsal: all ranks on cuda:0, hipIpc peer data
# plane, end-of-run digest guard): dense vs int8 + EF vs top-k at the given ratios, one run per seed, 23 rounds.
#   usage: bash tools/gpu_compress_sweep.sh <tag> "<seeds>" "<topk ratios>"
T=${1:-r5c}; SEEDS=${2:-"17 18 19"}; RATIOS=${3:-"0.10 0.20"}
R="FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 3"
args=()
for s in $SEEDS; do
  args+=("dense_s$s" 240 "$R --seed $s --json-out gpurun_out/$T/dense_s$s.json")
  args+=("int8_s$s" 240 "$R --seed $s --compress int8 --json-out gpurun_out/$T/int8_s$s.json")
  for r in $RATIOS; do
    args+=("topk${r}_s$s" 240 "$R --seed $s --compress topk --topk-ratio $r --json-out gpurun_out/$T/topk${r}_s$s.json")
  done
done
bash tools/gpu_steps.sh "$T" "${args[@]}"
