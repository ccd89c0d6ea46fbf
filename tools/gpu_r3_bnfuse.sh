#!/bin/bash
# BN-backward sums in the DGRAD epilogue: kernel + engine tests, ResNet-18 / MobileNet step A/B
# (FEDMI_CNN_FUSE_BN_BWD=0/1), rocprof step breakdown of the fused default; LeNet pipelined A/B bench.
set -u
O=gpurun_out/r3f
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
export TMPDIR=/tmp
STAGES="${STAGES:-tests bench prof pipe}"
for st in $STAGES; do
  case $st in
    tests)
      timeout -k 10 600 python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py -q -x \
        -k "fused_bn_sums or presummed or deterministic or tail_grads or emulated or trains_like or graph" \
        --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
      echo "tests rc=$rc" >> $S; tail -3 $O/tests.log >> $S; stop $rc ;;
    bench)
      for m in ${MODELS:-resnet18 mobilenet}; do
        for f in 0 1; do
          FEDMI_CNN_FUSE_BN_BWD=$f timeout -k 10 400 python bench.py --model $m --steps 3 --warmup 1 \
            --json-out $O/bench_${m}_f$f.json > $O/bench_${m}_f$f.log 2>&1; rc=$?
          echo "bench $m fuse=$f rc=$rc $(python -c "import json;r=json.load(open('$O/bench_${m}_f$f.json'));print(r['ms_per_step'],'ms/round',r['last_round'])" 2>&1)" >> $S
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
    pipe)
      for i in 1 2; do
        for pipe in 0 1; do
          FEDMI_LENET_PIPE=$pipe timeout -k 10 240 python bench.py --json-out $O/lenet_pipe${pipe}_$i.json \
            > $O/lenet_pipe${pipe}_$i.log 2>&1; rc=$?
          echo "lenet pipe=$pipe run=$i rc=$rc $(python -c "import json;d=json.load(open('$O/lenet_pipe${pipe}_$i.json'));print(d['rounds_per_sec'], d['ms_per_step'], d['last_round'])" 2>&1)" >> $S
          stop $rc
        done
      done ;;
  esac
done
echo done >> $S
