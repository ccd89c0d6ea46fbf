# round 6: deferred WGRAD reductions in the aten (zoo) backend -- bit-identity, kernel list, zoo A/B
bash tools/gpu_steps.sh r6_t \
  tests 600 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_kernel_list_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'deferred or launches or graph_replay or deterministic or fusion'" \
  zoo_on 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py densenet_cifar RegNetY_400MF DLA EfficientNetB0" \
  zoo_off 300 "env BENCH_MODES=native-graph FEDMI_WRED_DEFER=0 python -u tools/bench_hybrid.py densenet_cifar RegNetY_400MF DLA EfficientNetB0"
