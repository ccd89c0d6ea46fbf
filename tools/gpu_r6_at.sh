# round 6: 1x1 halo WGRAD kept to the CNN engine (aten backend: generic) -- tests + zoo / MobileNet check
M="densenet_cifar DPN26 SENet18 ResNeXt29_2x64d"
bash tools/gpu_steps.sh r6_at \
  kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'wgrad'" \
  zoot 400 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_kernel_list_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'deferred or launches or conv_fwd_bwd'" \
  mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
  zoo 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M"
