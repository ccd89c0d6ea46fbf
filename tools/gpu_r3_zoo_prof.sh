#!/bin/bash
# Zoo backend: per-kernel GPU time of graph-replayed steps (densenet_cifar, RegNetY_400MF) and the
# DPN26 / RegNetY / ShuffleNetG2 learning sweep vs fp32 (3 seeds x 2 lrs).
set -u
O=gpurun_out/r3zp
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
export TMPDIR=/tmp
STAGES="${STAGES:-prof gap}"
for st in $STAGES; do
  case $st in
    prof)
      for m in ${ZOO:-densenet_cifar RegNetY_400MF}; do
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- \
          python tools/prof_native_mode.py $m 13 > $O/prof_$m.log 2>&1; rc=$?
        echo "prof $m rc=$rc" >> $S; stop $rc
        tr=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
        python tools/zoo_step_kernels.py $tr 10 > $O/kernels_$m.txt 2>&1
        head -40 $O/kernels_$m.txt >> $S
        rm -f $tr
      done ;;
    bench)
      timeout -k 10 560 python tools/bench_hybrid.py ${ZOO:-densenet_cifar RegNetY_400MF} \
        > $O/bench_hybrid.jsonl 2> $O/bench_hybrid.err; rc=$?
      echo "bench rc=$rc" >> $S; cat $O/bench_hybrid.jsonl >> $S; stop $rc ;;
    gap)
      for lr in 0.02 0.005; do
        timeout -k 10 500 python tools/zoo_learning.py DPN26 RegNetY_400MF ShuffleNetG2 --seeds 0 1 2 --epochs 8 --lr $lr \
          >> $O/learning.jsonl 2>> $O/learning.err; rc=$?
        echo "gap lr=$lr rc=$rc" >> $S; stop $rc
      done ;;
  esac
done
echo done >> $S
