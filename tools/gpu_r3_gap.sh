#!/bin/bash
# DPN26 / RegNetY / ShuffleNetG2 native-vs-fp32 gaps: 3 seeds x 2 learning rates, 8 epochs each.
set -u
O=gpurun_out/r3g
mkdir -p $O
for lr in 0.02 0.005; do
  timeout -k 10 500 python tools/zoo_learning.py DPN26 RegNetY_400MF ShuffleNetG2 --seeds 0 1 2 --epochs 8 --lr $lr \
    >> $O/learning.jsonl 2>> $O/learning.err || exit $?
done
echo done
