#!/bin/bash
# Round-4 config 4 at 8 ranks: the bench.py --gpus 8 rehearsal (all ranks on cuda:0, hipIpc
# peer data plane, digest guard) for 23 rounds dense vs -c Y top-k at several ratios / dense warm-up vs int8.
T=${1:-r4t}
R="FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 3"
bash tools/gpu_steps.sh $T \
  dense 200 "$R --json-out gpurun_out/$T/reh8_dense.json" \
  topk1 200 "$R --compress topk --topk-ratio 0.01 --json-out gpurun_out/$T/reh8_topk.json" \
  int8 200 "$R --compress int8 --json-out gpurun_out/$T/reh8_int8.json" \
  topk1w2 200 "$R --compress topk --topk-ratio 0.01 --compress-warmup 2 --json-out gpurun_out/$T/reh8_topk_w2.json" \
  topk5 200 "$R --compress topk --topk-ratio 0.05 --json-out gpurun_out/$T/reh8_topk5.json" \
  topk10 200 "$R --compress topk --topk-ratio 0.10 --json-out gpurun_out/$T/reh8_topk10.json" \
  topk5w2 200 "$R --compress topk --topk-ratio 0.05 --compress-warmup 2 --json-out gpurun_out/$T/reh8_topk5_w2.json"
# N=8 projection with the per-round gap statistics, for the host-gap question
bash tools/gpu_steps.sh $T proj8 120 "python bench.py --breakdown --project-world 8 --steps 40 --warmup 5 --json-out gpurun_out/$T/proj8.json"
