# round 6: 1x1 WGRAD library route at <= 2048 pixels -- kernel test, MobileNet A/B (route on / off / on)
bash tools/gpu_steps.sh r6_m \
  test 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -k 'wgrad' -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  mbn_on 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  mbn_off 300 "env FEDMI_WGRAD_GEMM=0 python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  mbn_on2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
