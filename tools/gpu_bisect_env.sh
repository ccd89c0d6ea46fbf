#!/bin/bash
# Run one pytest selection under several environment settings (numerics bisection), each under its own time
# limit.  pytest exit 0 / 1 (passed / tests failed) continues; anything else (abort, fault, time limit) stops.
#   usage: bash tools/gpu_bisect_env.sh <tag> <seconds> <pytest selection> <env assignment>...   ("-" = none)
set -u
tag=$1; secs=$2; sel=$3; shift 3
out=gpurun_out/$tag
mkdir -p "$out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for envs in "$@"; do
  i=$((i + 1))
  [ "$envs" = "-" ] && envs=""
  echo "=== run $i env [$envs]" | tee -a "$out/summary.txt"
  env $envs timeout -k 10 "$secs" python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider $sel > "$out/run$i.log" 2>&1
  rc=$?
  echo "=== run $i rc=$rc $(tail -n1 "$out/run$i.log")" | tee -a "$out/summary.txt"
  grep -h "AssertionError: \|^E  " "$out/run$i.log" | head -3 | tee -a "$out/summary.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping (rc=$rc)" | tee -a "$out/summary.txt"; exit $rc; fi
done
exit 0
