# round 6: LeNet slow rounds 2-4 of the timed region -- vary the checkpoint writer's slots and the warmup
bash tools/gpu_steps.sh r6_af \
  s1 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 1" \
  s2 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 2" \
  s16 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 16" \
  w10 200 "python -u bench.py --breakdown --steps 30 --warmup 10" \
  noev 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --no-eval"
