# round 6: 1x1 halo WGRAD limited to small problems -- tests + A/B
bash tools/gpu_steps.sh r6_ar \
  kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'wgrad'" \
  eng 300 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'deterministic or deferred'" \
  mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
  goog_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model googlenet --steps 2 --warmup 1" \
  mbn2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  mbn_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model mobilenet --steps 3 --warmup 1"
