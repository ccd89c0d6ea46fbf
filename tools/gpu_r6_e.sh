# round 6: KS2 SGD operands loaded first (LeNet), then the c+d batch
bash tools/gpu_steps.sh r6_e \
  lenettest 300 "python -u -m pytest tests/test_lenet_kernels_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  bench_a 150 "python bench.py --json-out gpurun_out/r6_e/bench_a.json" \
  bench_b 150 "python bench.py --json-out gpurun_out/r6_e/bench_b.json" && bash tools/gpu_r6_d.sh && bash tools/gpu_r6_c.sh
