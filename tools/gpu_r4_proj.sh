#!/bin/bash
# Round-4: kernel tests touched by the top-k prune / BN ticket slots, then the 1-GPU projection of the N-client
# per-client round (bench.py --project-world N --breakdown) at N=1/2/4/8 and the 8-rank rehearsal with the guard.
T=${1:-r4p}
bash tools/gpu_steps.sh $T \
  tests 600 "python -u -m pytest tests/test_flat_ops_gpu.py tests/test_native_mode_gpu.py tests/test_eval_ckpt.py -x -q --timeout 200 --timeout-method thread" \
  proj1 120 "python bench.py --breakdown --steps 30 --warmup 5 --json-out gpurun_out/$T/proj1.json" \
  proj2 120 "python bench.py --breakdown --project-world 2 --steps 30 --warmup 5 --json-out gpurun_out/$T/proj2.json" \
  proj4 120 "python bench.py --breakdown --project-world 4 --steps 30 --warmup 5 --json-out gpurun_out/$T/proj4.json" \
  proj8 120 "python bench.py --breakdown --project-world 8 --steps 30 --warmup 5 --json-out gpurun_out/$T/proj8.json" \
  reh8 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 3 --json-out gpurun_out/$T/reh8.json"
