#!/bin/bash
# (1) rocprofv3 kernel stats of the -c Y kernels; (2) non-IID FedAvg seed/lr sweep, native vs fp32 engine.
set -u
O=gpurun_out/r3w
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
STAGES="${STAGES:-prof sweep}"
for st in $STAGES; do
  case $st in
    prof)
      export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o compress --output-format csv -- \
        python tools/bench_compress.py > $O/prof.log 2>&1; rc=$?
      echo "prof rc=$rc" >> $S; stop $rc
      find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/compress_kernel_stats.csv \; ;;
    sweep)
      for lr in 0.1 0.02; do
        for seed in 17 18 19; do
          for eng in native fp32; do
            timeout -k 10 300 python tools/fedavg_sim.py --model resnet18 --clients 2 --noniid 2 --rounds 6 \
              --engine $eng --lr $lr --seed $seed --out $O/sweep_${eng}_lr${lr}_s${seed}.jsonl > $O/sweep.log 2>&1; rc=$?
            echo "lr $lr seed $seed $eng rc=$rc $(tail -1 $O/sweep_${eng}_lr${lr}_s${seed}.jsonl | cut -c1-230)" >> $S
            stop $rc
          done
        done
      done ;;
  esac
done
echo done >> $S
