# round 6: fused -c Y int8 peer collective (test + timing), N>1 bench rehearsal with the split-eval compare loop,
# GoogLeNet kernel breakdown
o=gpurun_out/r6_d
mkdir -p $o
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_steps.sh r6_d \
  int8test 300 "python -u -m pytest tests/test_peer_comm_gpu.py -k 'int8 or abort' -x -v --timeout 240 --timeout-method thread -p no:cacheprovider" \
  peerbench 300 "python tools/bench_peer.py --world 2 4 --iters 200 --no-gate --out $o/peer_nogate.jsonl" \
  reh2 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --json-out $o/reh2.json" \
  reh4y 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 5 --warmup 2 --compress Y --json-out $o/reh4y.json" \
  googprof 300 "MODELS=googlenet bash tools/gpu_prof_models.sh r6_d/prof"
