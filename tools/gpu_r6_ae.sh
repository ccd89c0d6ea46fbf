# round 6: LeNet per-round device spans (where the mean round exceeds the median)
bash tools/gpu_steps.sh r6_ae \
  b1 200 "python -u bench.py --breakdown --steps 40 --warmup 3" \
  b2 200 "python -u bench.py --breakdown --steps 40 --warmup 3"
