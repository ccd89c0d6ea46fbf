#!/bin/bash
# Run named GPU steps, each under its own time limit, logging to gpurun_out/<tag>/.
# Any failing step ends the script right there: a failing GPU test may be a device fault (an illegal
# address surfaces as an ordinary pytest failure), and nothing more runs on the GPU after a fault.
#   usage: bash tools/gpu_steps.sh <tag> <name> <seconds> <command> [<name> <seconds> <command> ...]
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
while [ $# -ge 3 ]; do
  name=$1; secs=$2; cmd=$3; shift 3
  echo "=== $name (limit ${secs}s): $cmd" | tee -a "$out/steps.txt"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc wall=$(( $(date +%s) - start ))s" | tee -a "$out/steps.txt"
  tail -5 "$out/$name.log"
  if [ $rc -ne 0 ]; then
    echo "=== stopping after $name (rc=$rc)" | tee -a "$out/steps.txt"
    exit $rc
  fi
done
exit 0
