#!/bin/bash
# Iteration check: LeNet pipelined hand-off (tests + A/B bench), depthwise fused BN sums, native-backend
# determinism, MobileNet / ResNet-18 step with the fused BN-backward sums.
set -u
O=gpurun_out/r3i
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
export TMPDIR=/tmp
STAGES="${STAGES:-pipe tests bench}"
for st in $STAGES; do
  case $st in
    pipe)
      timeout -k 10 300 python -u -m pytest tests/test_lenet_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
        -k "pipelined or graph_epoch or sample_path or sgd" > $O/pipe_tests.log 2>&1; rc=$?
      echo "pipe tests rc=$rc" >> $S; tail -3 $O/pipe_tests.log >> $S; stop $rc
      for i in 1 2; do
        for pipe in 0 1; do
          FEDMI_LENET_PIPE=$pipe timeout -k 10 240 python bench.py --json-out $O/lenet_pipe${pipe}_$i.json \
            > $O/lenet_pipe${pipe}_$i.log 2>&1; rc=$?
          echo "lenet pipe=$pipe run=$i rc=$rc $(python -c "import json;d=json.load(open('$O/lenet_pipe${pipe}_$i.json'));print(d['rounds_per_sec'], d['ms_per_step'], d['last_round'])" 2>&1)" >> $S
          stop $rc
        done
      done ;;
    tests)
      timeout -k 10 600 python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_native_mode_gpu.py -q -x \
        -k "fused_bn_sums or presummed or backend_is_deterministic" \
        --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
      echo "tests rc=$rc" >> $S; tail -3 $O/tests.log >> $S; stop $rc ;;
    bench)
      for m in ${MODELS:-mobilenet resnet18}; do
        for f in 0 1; do
          FEDMI_CNN_FUSE_BN_BWD=$f timeout -k 10 400 python bench.py --model $m --steps 3 --warmup 1 \
            --json-out $O/bench_${m}_f$f.json > $O/bench_${m}_f$f.log 2>&1; rc=$?
          echo "bench $m fuse=$f rc=$rc $(python -c "import json;r=json.load(open('$O/bench_${m}_f$f.json'));print(r['ms_per_step'],'ms/round',r['last_round'])" 2>&1)" >> $S
          stop $rc
        done
      done ;;
  esac
done
echo done >> $S
