bash tools/gpu_steps.sh r6_a \
  bench 150 "python bench.py --json-out gpurun_out/r6_a/bench1.json" \
  r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/r6_a/r18.json" \
  mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/r6_a/mbn.json" \
  failover 600 "FEDMI_FAILOVER_REPORT=gpurun_out/r6_a/drills.jsonl python -u -m pytest tests/test_failover_kill.py -k 'client_sigkill and gpu' -x -v --timeout 420 --timeout-method thread -p no:cacheprovider"
