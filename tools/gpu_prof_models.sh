#!/bin/bash
# rocprofv3 kernel trace + stats of one ResNet-18 / MobileNet / LeNet FedAvg round each
# (bench.py, 1 timed round), each under its own time limit; stops at the first fault.
# The raw kernel trace is reduced on the box (per-kernel stats + one step's timeline) and deleted.
set -u
out=gpurun_out/${1:-pm}
mkdir -p "$out"
export TMPDIR=/tmp
for m in ${MODELS:-resnet18 mobilenet lenet}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/$m" -o run --output-format csv -- \
    python bench.py --model "$m" --steps 1 --warmup 1 > "$out/$m.log" 2>&1
  rc=$?
  echo "$m rc=$rc" >> "$out/summary.txt"
  [ $rc -eq 0 ] || exit $rc
  tr=$(find "$out/$m" -name '*kernel_trace.csv' | head -1)
  st=$(find "$out/$m" -name '*kernel_stats.csv' | head -1)
  [ -n "$st" ] && cp "$st" "$out/${m}_kernel_stats.csv"
  if [ "$m" != lenet ] && [ -n "$tr" ]; then
    python tools/prof_step.py "$tr" 300 > "$out/${m}_step.txt" 2>&1
  fi
  rm -rf "$out/$m"
done
