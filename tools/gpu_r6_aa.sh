# round 6: LeNet eval conv forward at 6 waves / SIMD (three workgroups per CU) -- tests + breakdown + stats
set -e
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/${TAG:-r6_aa}
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests/test_lenet_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -n 2 $out/tests.log
timeout -k 10 300 python3 bench.py --breakdown > $out/lenet_breakdown.log 2>&1
timeout -k 10 300 python3 bench.py > $out/lenet2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/lenet -o run -- python3 bench.py --steps 3 --warmup 1 > $out/lenet_prof.log 2>&1
st=$(find $out/lenet -name 'run_kernel_stats.csv' | head -n 1)
python3 tools/prof_summary.py "$st" lenet_sgd2 30 > $out/lenet_kernels.txt
rm -f $(find $out/lenet -name 'run_kernel_trace.csv')
grep "onv_fwd\|fc_eval" $out/lenet_kernels.txt || true
