# round 6: 1x1 halo WGRAD A/B beyond MobileNet -- MobileNetV2 (CNN engine) and the aten-backend zoo
M="densenet_cifar DenseNet121 DPN26 RegNetX_200MF RegNetY_400MF SimpleDLA EfficientNetB0 ResNeXt29_2x64d SENet18"
bash tools/gpu_steps.sh r6_as \
  mbv2 300 "python -u bench.py --model mobilenetv2 --steps 2 --warmup 1" \
  mbv2_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model mobilenetv2 --steps 2 --warmup 1" \
  zoo 400 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M" \
  zoo_off 400 "env BENCH_MODES=native-graph FEDMI_WGRAD_1X1=0 python -u tools/bench_hybrid.py $M"
