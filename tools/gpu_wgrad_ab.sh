#!/bin/bash
# A/B of the halo WGRAD vs the generic WGRAD (FEDMI_WGRAD_HALO) at the ResNet-18 batch-128 3x3 shapes,
# graph-replay timing + per-kernel stats.
set -u
out=gpurun_out/${1:-wab}
mkdir -p "$out"
export TMPDIR=/tmp
for v in "1 256" "0 0"; do
  set -- $v
  FEDMI_WGRAD_HALO=$1 FEDMI_WGRAD_HALO_WGS=$2 timeout -k 10 120 python tools/bench_tap.py --graph --iters 20 --batch 128 \
    --shapes l1,l2,l3,l4 --passes wgrad > "$out/tap_w$1_$2.log" 2>&1 || exit $?
  for sh in l1 l3; do
    FEDMI_WGRAD_HALO=$1 FEDMI_WGRAD_HALO_WGS=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/p_${sh}_w$1_$2" \
      -o run --output-format csv -- python tools/bench_tap.py --iters 20 --shapes $sh --passes wgrad \
      > "$out/p_${sh}_w$1_$2.txt" 2>&1 || exit $?
    rm -f "$out/p_${sh}_w$1_$2/run_kernel_trace.csv"
  done
done
echo done > "$out/done.txt"
