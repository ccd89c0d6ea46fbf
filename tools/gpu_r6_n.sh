# round 6: deferred WGRAD reductions (one wgrad_reduce_multi launch per step) -- bit-identity, kernel list, kernel
# tests, MobileNet / ResNet-18 A/B (FEDMI_WRED_DEFER=0 = per-conv reductions)
bash tools/gpu_steps.sh r6_n \
  tests 600 "python -u -m pytest tests/test_cnn_native_gpu.py tests/test_kernel_list_gpu.py tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --deselect tests/test_cnn_native_gpu.py::test_loss_and_tail_grads_match_torch --deselect tests/test_cnn_native_gpu.py::test_engine_is_deterministic" \
  mbn_on 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1 --breakdown" \
  mbn_off 300 "env FEDMI_WRED_DEFER=0 python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  r18_on 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1 --breakdown" \
  r18_off 300 "env FEDMI_WRED_DEFER=0 python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  mbn_on2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  r18_on2 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1"
