# round 6: GEN conv_tap A/B on the zoo trajectories, blocked maxpool3, fused int8 timing, GoogLeNet
o=gpurun_out/r6_g
mkdir -p $o
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_steps.sh r6_g \
  kern 400 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  dpn_gen0 300 "FEDMI_TAP_GEN=0 python -u -m pytest tests/test_native_mode_gpu.py -k 'family and DPN26' -x -q -s --timeout 280 --timeout-method thread -p no:cacheprovider" \
  dpn_gen1 300 "python -u -m pytest tests/test_native_mode_gpu.py -k 'family and DPN26' -x -q -s --timeout 280 --timeout-method thread -p no:cacheprovider" \
  zoo 600 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_cnn_native_gpu.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider" \
  peerbench 300 "python tools/bench_peer.py --world 2 4 --iters 200 --no-gate --out $o/peer_nogate.jsonl" \
  goog 300 "python bench.py --model googlenet --steps 2 --warmup 1 --json-out $o/goog.json" \
  goog_gen0 300 "FEDMI_TAP_GEN=0 python bench.py --model googlenet --steps 2 --warmup 1 --json-out $o/goog_gen0.json" \
  r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out $o/r18.json" \
  zoobench 400 "BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 DLA DPN26 PNASNetA > $o/zoo.jsonl" \
  zoobench0 400 "FEDMI_TAP_GEN=0 BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 DLA DPN26 PNASNetA > $o/zoo_gen0.jsonl" \
  googprof 300 "MODELS=googlenet bash tools/gpu_prof_models.sh r6_g/prof"
