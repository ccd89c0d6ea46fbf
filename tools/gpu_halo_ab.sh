#!/bin/bash
# A/B of conv_halo vs conv_tap (FEDMI_CONV_HALO) on the ResNet-18 3x3 shapes + one PMC pass each.
set -u
out=gpurun_out/${1:-hab}
mkdir -p "$out"
export TMPDIR=/tmp
for b in 128 32; do
  for h in 1 0; do
    FEDMI_CONV_HALO=$h timeout -k 10 120 python tools/bench_tap.py --iters 30 --batch $b --shapes l1,l2,l3,l4 \
      > "$out/tap_b${b}_h${h}.log" 2>&1 || exit $?
  done
done
for h in 1 0; do
  FEDMI_CONV_HALO=$h timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d "$out/pmc_h$h" -o run --output-format csv -- python tools/bench_tap.py --iters 3 --shapes l1,l2 > "$out/pmc_h$h.log" 2>&1 || exit $?
done
echo done > "$out/done.txt"
