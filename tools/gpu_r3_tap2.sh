#!/bin/bash
# conv_tap with 2 LDS stages (FEDMI_TAP_STAGES=2: one more workgroup per CU) vs 3: kernel tests under the
# variant, per-shape graph timings, ResNet-18 / VGG11 round A/B.
set -u
O=gpurun_out/r3t
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
export TMPDIR=/tmp
FEDMI_TAP_STAGES=2 timeout -k 10 500 python -u -m pytest tests/test_cnn_kernels_gpu.py -q -x -k "conv or dgrad or resnet18" \
  --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests(stages=2) rc=$rc" >> $S; tail -2 $O/tests.log >> $S; stop $rc
for ns in 3 2; do
  FEDMI_TAP_STAGES=$ns timeout -k 10 120 python tools/bench_tap.py --graph --iters 20 --batch 128 --shapes l1,l2,l3,l4,d2,d4 \
    > $O/tap_s$ns.jsonl 2>&1; rc=$?
  echo "tap stages=$ns rc=$rc" >> $S; grep -v amdgpu $O/tap_s$ns.jsonl | grep -E "fwd_stats|dgrad_tap" >> $S; stop $rc
done
for m in resnet18 vgg11; do
  for ns in 3 2; do
    FEDMI_TAP_STAGES=$ns timeout -k 10 400 python bench.py --model $m --steps 3 --warmup 1 --json-out $O/bench_${m}_s$ns.json \
      > $O/bench_${m}_s$ns.log 2>&1; rc=$?
    echo "bench $m stages=$ns rc=$rc $(python -c "import json;r=json.load(open('$O/bench_${m}_s$ns.json'));print(r['ms_per_step'],'ms/round')" 2>&1)" >> $S
    stop $rc
  done
done
echo done >> $S
