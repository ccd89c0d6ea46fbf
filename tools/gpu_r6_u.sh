# round 6: zoo A/B of the round-6 routing changes (GEN DGRAD, library 1x1 WGRAD) on the aten backend
M="densenet_cifar DenseNet121 DPN26 RegNetX_200MF SimpleDLA"
bash tools/gpu_steps.sh r6_u \
  base 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M" \
  nodgen 300 "env BENCH_MODES=native-graph FEDMI_DGRAD_GEN=0 python -u tools/bench_hybrid.py $M" \
  nolib 300 "env BENCH_MODES=native-graph FEDMI_WGRAD_GEMM=0 python -u tools/bench_hybrid.py $M" \
  base2 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M"
