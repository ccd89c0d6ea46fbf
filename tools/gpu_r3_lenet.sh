#!/bin/bash
# LeNet eval overlap + top-k launches: tests, compression timings, bench A/B (overlap on/off, 2 runs each).
set -u
O=gpurun_out/r3l
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
export TMPDIR=/tmp
STAGES="${STAGES:-tests compress bench}"
for st in $STAGES; do
  case $st in
    tests)
      timeout -k 10 500 python -u -m pytest tests/test_flat_ops_gpu.py tests/test_lenet_kernels_gpu.py tests/test_system_gpu.py -q -x \
        --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
      echo "tests rc=$rc" >> $S; tail -3 $O/tests.log >> $S; stop $rc ;;
    compress)
      timeout -k 10 300 python tools/bench_compress.py $O/compress.jsonl > $O/compress.log 2>&1; rc=$?
      echo "compress rc=$rc" >> $S; cat $O/compress.log >> $S; stop $rc ;;
    bench)
      for i in 1 2; do
        for ov in 0 1; do
          FEDMI_LENET_EVAL_OVERLAP=$ov timeout -k 10 240 python bench.py --json-out $O/lenet_ov${ov}_$i.json \
            > $O/lenet_ov${ov}_$i.log 2>&1; rc=$?
          echo "lenet overlap=$ov run=$i rc=$rc $(python -c "import json;d=json.load(open('$O/lenet_ov${ov}_$i.json'));print(d['rounds_per_sec'], d['ms_per_step'], d['last_round'])" 2>&1)" >> $S
          stop $rc
        done
      done ;;
  esac
done
echo done >> $S
