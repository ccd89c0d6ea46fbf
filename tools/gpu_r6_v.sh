# round 6: zoo after restricting the GEN DGRAD / library WGRAD routes to the CNN engine; deferral on / off
M="densenet_cifar DenseNet121 DPN26 RegNetX_200MF SimpleDLA RegNetY_400MF EfficientNetB0"
bash tools/gpu_steps.sh r6_v \
  tests 600 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_kernel_list_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'deferred or launches or graph_replay or deterministic or fusion or conv_fwd_bwd'" \
  on 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M" \
  off 300 "env BENCH_MODES=native-graph FEDMI_WRED_DEFER=0 python -u tools/bench_hybrid.py $M" \
  on2 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M"
