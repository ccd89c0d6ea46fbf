# round 6: 1x1 WGRAD on conv_wgrad_halo<1, 1> -- kernel tests, engine bit-identity tests, A/B (FEDMI_WGRAD_1X1=0)
bash tools/gpu_steps.sh r6_ap \
  kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'wgrad or dgrad'" \
  eng 300 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'deterministic or deferred'" \
  mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  mbn_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
  goog_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model googlenet --steps 2 --warmup 1" \
  r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  mbn2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
