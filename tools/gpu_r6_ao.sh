# round 6: final N>1 rehearsal of bench.py on one GPU (ranks time-slice the card; peer transport verified vs gloo)
o=gpurun_out/r6_ao
mkdir -p $o
bash tools/gpu_steps.sh r6_ao \
  reh2 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 5 --warmup 2 --json-out $o/reh2.json" \
  reh4 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 4 --steps 5 --warmup 2 --json-out $o/reh4.json"
