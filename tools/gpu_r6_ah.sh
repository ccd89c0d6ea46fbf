# round 6: bench.py with the 2-slot checkpoint writer default
bash tools/gpu_steps.sh r6_ah \
  def 200 "python -u bench.py" \
  def2 200 "python -u bench.py" \
  w1 200 "python -u bench.py --warmup 1 --steps 20 --breakdown" \
  k50 200 "python -u bench.py --warmup 2 --steps 50 --breakdown"
