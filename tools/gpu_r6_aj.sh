# round 6: CNN benches with the 2-slot checkpoint writer default (vs 4)
bash tools/gpu_steps.sh r6_aj \
  r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1 --breakdown" \
  r18_s4 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1 --ckpt-slots 4 --breakdown" \
  mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1 --breakdown" \
  mbn_s4 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1 --ckpt-slots 4 --breakdown"
