#!/bin/bash
# Round-4 N>1 readiness on ONE GPU:
#  guard   - bench.py's end-of-run digest guard passes a correct 2-rank rehearsal and fires on an injected
#            skipped FedAvg (tests/test_bench_guard_gpu.py)
#  projN   - bench.py --project-world N --breakdown: one client runs rank 0's 1/N share of the round (train
#            shard, eval shard, checkpoint writer), no collective -- per-client critical path at N=1/2/4/8
#  peer8   - 8-process hipIpc all-reduce at 248 KB / 44.7 MB (all ranks on cuda:0: time-sliced, not xGMI)
#  reh8    - 8-rank rehearsal of bench.py --gpus 8 with the digest guard
T=${1:-r4s}
bash tools/gpu_steps.sh $T \
  guard 200 "python -u -m pytest tests/test_bench_guard_gpu.py -x -v --timeout 150 --timeout-method thread" \
  proj1 120 "python bench.py --breakdown --steps 30 --warmup 3 --json-out gpurun_out/$T/proj1.json" \
  proj2 120 "python bench.py --breakdown --project-world 2 --steps 30 --warmup 3 --json-out gpurun_out/$T/proj2.json" \
  proj4 120 "python bench.py --breakdown --project-world 4 --steps 30 --warmup 3 --json-out gpurun_out/$T/proj4.json" \
  proj8 120 "python bench.py --breakdown --project-world 8 --steps 30 --warmup 3 --json-out gpurun_out/$T/proj8.json" \
  peer8 200 "python tools/bench_peer.py --world 2 8 --iters 200 --out gpurun_out/$T/peer.jsonl" \
  reh8 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 3 --json-out gpurun_out/$T/reh8.json"
