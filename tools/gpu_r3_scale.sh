#!/bin/bash
# Round-3 N=8 readiness on ONE GPU: 8-process peer collectives, the RCCL lifecycle at world 1,
# the checkpoint writer at the 8-client cadence, bench N=1, and an 8-rank gloo rehearsal of
# bench.py (FEDMI_BENCH_REHEARSE=1: every rank on cuda:0 -- a launch/correctness test, not a
# scaling number).  Every GPU step has its own limit; a crash-class exit stops the script.
set -u
mkdir -p gpurun_out/r3s
S=gpurun_out/r3s/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
STAGES="${STAGES:-tests writer bench reh8}"
for st in $STAGES; do
  case $st in
    tests) timeout -k 10 500 python -u -m pytest tests/test_peer_comm_gpu.py tests/test_rccl_gpu.py -x -v \
             --timeout 220 --timeout-method thread > gpurun_out/r3s/tests.log 2>&1; rc=$?
           echo "tests rc=$rc" >> $S; tail -4 gpurun_out/r3s/tests.log >> $S; stop $rc ;;
    writer) timeout -k 10 200 python tools/bench_ckpt_writer.py --rounds 1000 --out gpurun_out/r3s/ckpt_writer.jsonl \
             > gpurun_out/r3s/writer.log 2>&1; rc=$?
           echo "writer rc=$rc" >> $S; cat gpurun_out/r3s/writer.log >> $S; stop $rc ;;
    bench) timeout -k 10 300 python bench.py --json-out gpurun_out/r3s/bench1.json > gpurun_out/r3s/bench1.log 2>&1; rc=$?
           echo "bench rc=$rc" >> $S; tail -2 gpurun_out/r3s/bench1.log >> $S; stop $rc ;;
    reh8) FEDMI_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 \
             --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 3 \
             --json-out gpurun_out/r3s/reh8.json > gpurun_out/r3s/reh8.log 2>&1; rc=$?
           echo "reh8 rc=$rc" >> $S; tail -3 gpurun_out/r3s/reh8.log >> $S; stop $rc ;;
  esac
done
echo done >> $S
