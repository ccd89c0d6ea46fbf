#!/bin/bash
# Iteration check: fused BN-backward sums (prefetched epilogues) and side-stream weight gradients:
# kernel / engine tests, then ResNet-18 / MobileNet step A/B over FEDMI_CNN_FUSE_BN_BWD x FEDMI_CNN_WGRAD_STREAM,
# rocprof step breakdown of the default.
set -u
O=gpurun_out/r3i
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
export TMPDIR=/tmp
STAGES="${STAGES:-tests bench prof}"
for st in $STAGES; do
  case $st in
    tests)
      timeout -k 10 600 python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py -q -x \
        -k "fused_bn_sums or presummed or deterministic or tail_grads or graph or splitk or accumulate or residual" \
        --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
      echo "tests rc=$rc" >> $S; tail -3 $O/tests.log >> $S; stop $rc ;;
    bench)
      for m in ${MODELS:-resnet18 mobilenet}; do
        for cfg in "0 0" "1 0" "0 1" "1 1"; do
          set -- $cfg
          FEDMI_CNN_FUSE_BN_BWD=$1 FEDMI_CNN_WGRAD_STREAM=$2 timeout -k 10 400 python bench.py --model $m --steps 3 --warmup 1 \
            --json-out $O/bench_${m}_f$1s$2.json > $O/bench_${m}_f$1s$2.log 2>&1; rc=$?
          echo "bench $m fuse=$1 stream=$2 rc=$rc $(python -c "import json;r=json.load(open('$O/bench_${m}_f$1s$2.json'));print(r['ms_per_step'],'ms/round',r['last_round'])" 2>&1)" >> $S
          stop $rc
        done
      done ;;
    prof)
      for m in ${MODELS:-resnet18 mobilenet}; do
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- \
          python bench.py --model $m --steps 1 --warmup 1 > $O/prof_$m.log 2>&1; rc=$?
        echo "prof $m rc=$rc" >> $S; stop $rc
        tr=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
        python tools/step_breakdown.py $tr 30 40 --json $O/breakdown_$m.json > $O/breakdown_$m.txt 2>&1
        cat $O/breakdown_$m.txt >> $S
        python tools/prof_step.py $tr 40 > $O/timeline_$m.txt 2>&1
        rm -f $tr
      done ;;
  esac
done
echo done >> $S
