# round 6: HEAD kernel breakdowns after the deferred WGRAD reductions (MobileNet, ResNet-18)
set -e
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/r6_p
mkdir -p $out
for m in mobilenet resnet18; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$m -o run -- python3 bench.py --model $m --steps 1 --warmup 1 > $out/${m}_bench.log 2>&1
  tr=$(find $out/$m -name 'run_kernel_trace.csv' | head -n 1)
  st=$(find $out/$m -name 'run_kernel_stats.csv' | head -n 1)
  python3 tools/prof_summary.py "$st" sched_next 40 > $out/${m}_kernels.txt
  python3 tools/prof_step.py "$tr" 300 > $out/${m}_step.txt
  rm -f "$tr"
  tail -n 2 $out/${m}_step.txt
done
