#!/bin/bash
# ResNet-18 FedAvg, 2 clients rehearsed on ONE GPU (gloo data plane): IID strided split vs non-IID
# label shards (2 shards per client, McMahan et al.), same rounds, test accuracy per round.
#   bash tools/noniid_gpu.sh <out_dir> [rounds]
set -u
out=$1; rounds=${2:-8}
mkdir -p "$out"
export FEDMI_BENCH_REHEARSE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
for split in iid noniid; do
  extra=""; [ "$split" = noniid ] && extra="--noniid 2"
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --model resnet18 --gpus 2 --steps "$rounds" --warmup 1 \
    --eval-full $extra --json-out "$out/resnet18_2c_$split.json" > "$out/resnet18_2c_$split.log" 2>&1 || exit $?
done
