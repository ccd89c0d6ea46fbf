# round 6: product-path refresh (bench_system.py: server.py primary + backup + client.py processes over gRPC)
bash tools/gpu_steps.sh r6_ac \
  lenet1 300 "python -u bench_system.py --clients 1 --rounds 60 --warmup 10 --json-out gpurun_out/r6_ac/lenet1.json" \
  lenet2 300 "python -u bench_system.py --clients 2 --rounds 60 --warmup 10 --json-out gpurun_out/r6_ac/lenet2.json" \
  mbn2 400 "python -u bench_system.py --clients 2 --model mobilenet --rounds 10 --warmup 3 --json-out gpurun_out/r6_ac/mbn2.json"
