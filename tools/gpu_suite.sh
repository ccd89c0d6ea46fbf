#!/bin/bash
# Validation set on one GPU box (each step under its own time limit, a fault / abort / time limit ends the run):
#   suite  - every GPU test (pytest -m gpu), thread-timeout per test
#   smoke  - __graft_entry__.smoke()
#   bench  - the headline bench (LeNet FedAvg, 1 GPU) + ResNet-18 / MobileNet FedAvg rounds
#   usage: bash tools/gpu_suite.sh <tag> [stages]      stages: any of "suite smoke bench" (default all)
T=${1:-suite}; STAGES=${2:-"suite smoke bench"}
args=()
for st in $STAGES; do
  case $st in
    suite) args+=(suite 1100 "python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider") ;;
    smoke) args+=(smoke 180 "python -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench) args+=(bench 150 "python bench.py --json-out gpurun_out/$T/bench1.json"
                  r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/$T/r18.json"
                  mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/$T/mbn.json") ;;
  esac
done
bash tools/gpu_steps.sh "$T" "${args[@]}"
