# round 6: LeNet headline at HEAD (x2) + GoogLeNet kernel breakdown after the GEN DGRAD
set -e
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/r6_s
mkdir -p $out
timeout -k 10 300 python3 bench.py > $out/lenet1.log 2>&1
timeout -k 10 300 python3 bench.py > $out/lenet2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/googlenet -o run -- python3 bench.py --model googlenet --steps 1 --warmup 1 > $out/googlenet_prof.log 2>&1
tr=$(find $out/googlenet -name 'run_kernel_trace.csv' | head -n 1)
st=$(find $out/googlenet -name 'run_kernel_stats.csv' | head -n 1)
python3 tools/prof_summary.py "$st" sched_next 50 > $out/googlenet_kernels.txt
python3 tools/prof_step.py "$tr" 300 > $out/googlenet_step.txt
rm -f "$tr"
tail -n 1 $out/googlenet_step.txt
