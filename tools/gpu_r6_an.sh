# round 6: split-K combine with 4 splits' loads in flight per step (vs 2) -- tests + A/B
bash tools/gpu_steps.sh r6_an \
  kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'conv or fused or tap'" \
  r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  r18b 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
  goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
  mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
