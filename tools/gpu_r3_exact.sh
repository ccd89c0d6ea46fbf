#!/bin/bash
# Which native-mode change breaks fused == unfused bit-identity on densenet_cifar: the test under each switch.
set -u
O=gpurun_out/r3e
mkdir -p $O
S=$O/summary.txt
for v in "1 1 1" "0 0 0" "1 0 1" "0 1 1" "1 1 0"; do
  set -- $v
  FEDMI_ZOO_FAST=$1 FEDMI_NATIVE_CACHE=$2 FEDMI_BN_ROWS_FUSED=$3 timeout -k 10 300 python -u -m pytest \
    tests/test_native_mode_gpu.py -q -x -k "fusion_is_exact or backend_is_deterministic" --timeout 240 --timeout-method thread \
    > $O/t_$1$2$3.log 2>&1; rc=$?
  echo "fast=$1 cache=$2 rowsfused=$3 rc=$rc $(tail -1 $O/t_$1$2$3.log)" >> $S
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 400 python tools/bench_hybrid.py densenet_cifar RegNetY_400MF > $O/bench.jsonl 2> $O/bench.err; rc=$?
echo "bench rc=$rc" >> $S; cat $O/bench.jsonl >> $S
echo done >> $S
