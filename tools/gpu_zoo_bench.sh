#!/bin/bash
# One full FedAvg round per zoo model on 1 GPU (bench.py JSON lines), plus the BASELINE side configs
# (-c Y top-k compression on LeNet, non-IID ResNet-18).  Each step has its own time limit; a crash-class
# exit stops the script.
set -u
mkdir -p gpurun_out/benches
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "gpurun_out/benches/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $(grep -o '"rounds_per_sec": [0-9.]*' gpurun_out/benches/$name.log)" >> gpurun_out/benches/summary.txt
  if [ $rc -ge 124 ]; then echo "STOP $name $rc" >> gpurun_out/benches/summary.txt; exit $rc; fi
}
run lenet_topk 200 --compress topk --topk-ratio 0.01
run lenet_int8 200 --compress int8
run resnet18_noniid 300 --model resnet18 --noniid 2 --steps 2 --warmup 1
for m in ${MODELS:-resnext29_2x64d senet18 dla efficientnetb0 densenet121 dpn26 simpledla}; do
  run "$m" 300 --model "$m" --steps 1 --warmup 1
done
echo done >> gpurun_out/benches/summary.txt
