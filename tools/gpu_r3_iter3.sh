#!/bin/bash
set -u
O=gpurun_out/r3k
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
export TMPDIR=/tmp
timeout -k 10 200 python tools/diag_topk_system.py > $O/diag_topk.log 2>&1; rc=$?
echo "diag rc=$rc" >> $S; grep -E "round|tail|flag" $O/diag_topk.log >> $S; stop $rc
timeout -k 10 400 python -u -m pytest tests/test_system_gpu.py tests/test_flat_ops_gpu.py -q -x --timeout 240 --timeout-method thread \
  > $O/sys_tests.log 2>&1; rc=$?
echo "system+flat tests rc=$rc" >> $S; tail -3 $O/sys_tests.log >> $S; stop $rc
timeout -k 10 800 python -u -m pytest tests/test_native_mode_gpu.py -q -x --timeout 300 --timeout-method thread \
  > $O/nm_tests.log 2>&1; rc=$?
echo "native-mode tests rc=$rc" >> $S; tail -3 $O/nm_tests.log >> $S; stop $rc
timeout -k 10 560 python tools/bench_hybrid.py densenet_cifar RegNetY_400MF DenseNet121 \
  > $O/bench_hybrid.jsonl 2> $O/bench_hybrid.err; rc=$?
echo "bench rc=$rc" >> $S; cat $O/bench_hybrid.jsonl >> $S; stop $rc
echo done >> $S
