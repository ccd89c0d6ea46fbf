#!/bin/bash
# CNN engines after the channel-chunked BN applies: tests, bench step times, rocprof step breakdowns.
set -u
O=gpurun_out/r3c
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
export TMPDIR=/tmp
STAGES="${STAGES:-tests bench prof compress}"
for st in $STAGES; do
  case $st in
    tests)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py tests/test_flat_ops_gpu.py} -q -x \
        --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
      echo "tests rc=$rc" >> $S; tail -3 $O/tests.log >> $S; stop $rc ;;
    bench)
      for m in ${MODELS:-resnet18 mobilenet mobilenetv2}; do
        timeout -k 10 400 python bench.py --model $m --steps 3 --warmup 1 --json-out $O/bench_$m.json > $O/bench_$m.log 2>&1; rc=$?
        echo "bench $m rc=$rc $(python -c "import json;r=json.load(open('$O/bench_$m.json'));print(r['ms_per_step'],'ms/round',r['last_round'])" 2>&1)" >> $S
        stop $rc
      done ;;
    prof)
      for m in ${MODELS:-resnet18 mobilenet mobilenetv2}; do
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- \
          python bench.py --model $m --steps 1 --warmup 1 > $O/prof_$m.log 2>&1; rc=$?
        echo "prof $m rc=$rc" >> $S; stop $rc
        tr=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
        python tools/step_breakdown.py $tr 30 40 --json $O/breakdown_$m.json > $O/breakdown_$m.txt 2>&1
        cat $O/breakdown_$m.txt >> $S
        python tools/prof_step.py $tr 40 > $O/timeline_$m.txt 2>&1
        rm -f $tr
      done ;;
    compress)
      timeout -k 10 300 python tools/bench_compress.py $O/compress.jsonl > $O/compress.log 2>&1; rc=$?
      echo "compress rc=$rc" >> $S; cat $O/compress.log >> $S; stop $rc ;;
  esac
done
echo done >> $S
