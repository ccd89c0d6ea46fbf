# round 6: LeNet epoch graph double-instanced (alternate launches) -- slow-round check at 4 / 16 slots and default
bash tools/gpu_steps.sh r6_ai \
  s4 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 4" \
  s16 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 16" \
  w1 200 "python -u bench.py --warmup 1 --steps 20 --breakdown" \
  def 200 "python -u bench.py"
