#!/bin/bash
# Round 3: re-run of the fp64-stats kernel tests, the fused top-k, and a traced non-IID rehearsal.
set -u
O=gpurun_out/r3f
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
STAGES="${STAGES:-tests compress noniid}"
for st in $STAGES; do
  case $st in
    tests)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py} \
        tests/test_flat_ops_gpu.py -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
      echo "tests rc=$rc" >> $S; grep -E "FAILED|passed|failed" $O/tests.log | tail -12 >> $S; stop $rc ;;
    compress)
      timeout -k 10 300 python tools/bench_compress.py $O/compress.jsonl > $O/compress.log 2>&1; rc=$?
      echo "compress rc=$rc" >> $S; cat $O/compress.log >> $S; stop $rc ;;
    noniid)
      export FEDMI_BENCH_REHEARSE=1
      for eng in native fp32; do
        env_extra=""; [ "$eng" = fp32 ] && export FEDMI_TORCH_PATH=1 || unset FEDMI_TORCH_PATH
        timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
          --master-port $((29500 + RANDOM % 1000)) bench.py --model resnet18 --gpus 2 --steps 3 --warmup 1 \
          --eval-full --noniid 2 --trace --json-out $O/noniid_$eng.json > $O/noniid_$eng.log 2>&1; rc=$?
        echo "bench noniid $eng rc=$rc" >> $S; grep trace $O/noniid_$eng.log >> $S; stop $rc
      done ;;
  esac
done
echo done >> $S
