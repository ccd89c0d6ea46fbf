# round 6: BN-backward reduce with two rows' loads in flight (bit-identical) -- tests + A/B
bash tools/gpu_steps.sh r6_am \
  kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'bn'" \
  eng 300 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'deterministic'" \
  goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
  mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  goog2 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
  mbn2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
