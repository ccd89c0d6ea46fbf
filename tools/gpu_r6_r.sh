# round 6: stride-1 DGRAD on conv_tap<GEN> (O % 8 from 16 channels) -- kernel tests, GoogLeNet engine tests, GoogLeNet A/B
bash tools/gpu_steps.sh r6_r \
  kern 400 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  eng 400 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'GoogLeNet or deferred'" \
  goog_on 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
  goog_off 300 "env FEDMI_TAP_GEN=0 python -u bench.py --model googlenet --steps 2 --warmup 1" \
  zoo 500 "python -u -m pytest tests/test_native_mode_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'not family'"
