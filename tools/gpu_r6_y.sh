# round 6: defer only small WGRAD partial sets (FEDMI_WRED_DEFER_MB), reversed reduce order -- A/B + bit-identity
bash tools/gpu_steps.sh r6_y \
  test 400 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k deferred" \
  r18_8 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  r18_all 300 "env FEDMI_WRED_DEFER_MB=100000 python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  r18_64 300 "env FEDMI_WRED_DEFER_MB=64 python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  mbn_8 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  mbn_all 300 "env FEDMI_WRED_DEFER_MB=100000 python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  r18_8b 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  goog_8 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
  goog_all 300 "env FEDMI_WRED_DEFER_MB=100000 python -u bench.py --model googlenet --steps 2 --warmup 1"
