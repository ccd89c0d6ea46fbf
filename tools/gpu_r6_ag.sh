# round 6: checkpoint writer slots touched at construction -- the slow rounds 2-4 should be gone
bash tools/gpu_steps.sh r6_ag \
  d4 200 "python -u bench.py --breakdown --steps 30 --warmup 3" \
  s16 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 16" \
  def 200 "python -u bench.py" \
  def2 200 "python -u bench.py"
