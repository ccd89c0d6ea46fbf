#!/bin/bash
# Native aten backend with BN/ReLU fusion: GPU tests + per-step times vs fp32 and unfused.
set -u
O=gpurun_out/r3z
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
STAGES="${STAGES:-tests bench}"
for st in $STAGES; do
  case $st in
    tests)
      timeout -k 10 560 python -u -m pytest tests/test_native_mode_gpu.py -q -x --timeout 300 --timeout-method thread \
        > $O/tests.log 2>&1; rc=$?
      echo "tests rc=$rc" >> $S; tail -4 $O/tests.log >> $S; stop $rc ;;
    bench)
      timeout -k 10 560 python tools/bench_hybrid.py ${ZOO:-densenet_cifar DenseNet121 RegNetY_400MF SENet18 DPN26 DLA ResNeXt29_2x64d EfficientNetB0 ShuffleNetG2} \
        > $O/bench_hybrid.jsonl 2> $O/bench_hybrid.err; rc=$?
      echo "bench rc=$rc" >> $S; cat $O/bench_hybrid.jsonl >> $S; stop $rc ;;
  esac
done
echo done >> $S
