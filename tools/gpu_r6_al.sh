# round 6: split-K FWD/DGRAD combine with 2 splits' loads in flight per step (bit-identical) -- tests + A/B
bash tools/gpu_steps.sh r6_al \
  kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'conv or fused or tap'" \
  r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  r18b 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
  mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
