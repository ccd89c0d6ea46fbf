T=r4s2
bash tools/gpu_steps.sh $T \
  sys 400 "python -u -m pytest tests/test_system_gpu.py tests/test_failover_collective.py -x -v --timeout 200 --timeout-method thread -m gpu" \
  proj8 120 "python bench.py --breakdown --project-world 8 --steps 20 --warmup 3 --json-out gpurun_out/$T/proj8.json" \
  proj1 120 "python bench.py --breakdown --steps 20 --warmup 3 --json-out gpurun_out/$T/proj1.json" \
  prof8 200 "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/$T/prof8 -o p -- python \$GRAFT_REPO_ROOT/bench.py --project-world 8 --steps 20 --warmup 3"
