#!/bin/bash
# A/B of conv_halo vs conv_tap (FEDMI_CONV_HALO) on the ResNet-18 3x3 shapes, graph-replay timing,
# plus conv_halo phase stamps.
set -u
out=gpurun_out/${1:-hab}
mkdir -p "$out"
export TMPDIR=/tmp
for b in 128; do
  for h in 1 0; do
    FEDMI_CONV_HALO=$h timeout -k 10 120 python tools/bench_tap.py --graph --iters 20 --batch $b --shapes l1,l2,l3,l4 \
      > "$out/tap_b${b}_h${h}.log" 2>&1 || exit $?
  done
done
FEDMI_CONV_HALO=1 FEDMI_HALO_DEEP64=1 timeout -k 10 120 python tools/bench_tap.py --graph --iters 20 --shapes l1 \
  > "$out/tap_b128_h1_deep64.log" 2>&1 || exit $?
timeout -k 10 120 python tools/halo_stamps.py --batch 128 > "$out/stamps_b128.log" 2>&1 || exit $?
timeout -k 10 120 python tools/halo_stamps.py --batch 128 --split --shapes l3,l4 > "$out/stamps_b128_split.log" 2>&1 || exit $?
FEDMI_HALO_DEEP64=1 timeout -k 10 120 python tools/halo_stamps.py --batch 128 --shapes l1 > "$out/stamps_b128_deep64.log" 2>&1 || exit $?
echo done > "$out/done.txt"
