#!/bin/bash
# Round-4 LeNet two-launch path after the prune: kernel tests, host-ASan driver, smoke, bench,
# N=8 projection with per-phase mean/max, and the -c Y top-k ratio 0.2 rehearsal.
T=${1:-r4l}
bash tools/gpu_steps.sh $T \
  tests 400 "python -u -m pytest tests/test_lenet_kernels_gpu.py tests/test_kernel_list_gpu.py tests/test_eval_ckpt.py tests/test_cnn_kernels_gpu.py -x -v --timeout 200 --timeout-method thread" \
  asan 120 "ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0 ./tools/asan/bin/lenet_engine_asan" \
  smoke 120 "python -c 'import __graft_entry__ as g; g.smoke()'" \
  bench 120 "python bench.py --json-out gpurun_out/$T/bench1.json" \
  proj8 120 "python bench.py --breakdown --project-world 8 --steps 40 --warmup 5 --json-out gpurun_out/$T/proj8.json" \
  topk20 200 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 3 --compress topk --topk-ratio 0.2 --json-out gpurun_out/$T/reh8_topk20.json"
