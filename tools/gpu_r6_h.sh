# round 6: GEN conv_tap correctness sweep + zoo A/B (FEDMI_TAP_GEN=0 vs default), GoogLeNet A/B, int8 timing
o=gpurun_out/r6_h
mkdir -p $o
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_steps.sh r6_h \
  sweep 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -k 'gen_sweep or maxpool3' -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  zoobench 400 "BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 DLA DPN26 PNASNetA > $o/zoo.jsonl" \
  zoobench0 400 "FEDMI_TAP_GEN=0 BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 DLA DPN26 PNASNetA > $o/zoo_gen0.jsonl" \
  goog 300 "python bench.py --model googlenet --steps 2 --warmup 1 --json-out $o/goog.json" \
  goog_gen0 300 "FEDMI_TAP_GEN=0 python bench.py --model googlenet --steps 2 --warmup 1 --json-out $o/goog_gen0.json" \
  peerbench 300 "python tools/bench_peer.py --world 2 4 --iters 200 --no-gate --out $o/peer_nogate.jsonl" \
  fam_gen0 400 "FEDMI_TAP_GEN=0 python -u -m pytest tests/test_native_mode_gpu.py -k 'family' -q -s --timeout 380 --timeout-method thread -p no:cacheprovider" \
  fam_gen1 400 "python -u -m pytest tests/test_native_mode_gpu.py -k 'family' -q -s --timeout 380 --timeout-method thread -p no:cacheprovider"
