# round 6: N=8 per-client projection (1 GPU, rank 0's shard, full eval) with the round breakdown
bash tools/gpu_steps.sh r6_ak \
  p8 200 "python -u bench.py --project-world 8 --steps 100 --warmup 5 --breakdown" \
  p8b 200 "python -u bench.py --project-world 8 --steps 100 --warmup 5"
