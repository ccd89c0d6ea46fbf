# round 6: config-3 gate after the one-sided change + smoke
bash tools/gpu_steps.sh r6_x \
  config3 400 "python -u -m pytest tests/test_noniid_gpu.py -x -q -s --timeout 380 --timeout-method thread -p no:cacheprovider -k config3" \
  smoke 120 "python -c 'import __graft_entry__ as g; g.smoke()'" && \
bash tools/gpu_steps.sh r6_x2 \
  vgg 300 "python -u bench.py --model vgg16 --steps 3 --warmup 1" \
  preact 300 "python -u bench.py --model preactresnet18 --steps 3 --warmup 1" \
  mbv2 300 "python -u bench.py --model mobilenetv2 --steps 3 --warmup 1"
