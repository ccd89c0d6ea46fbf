#!/bin/bash
# Round 3: fp64 BN accumulation (determinism) + peer gating: GPU tests, parity diagnostic, non-IID bench rehearsal.
set -u
O=gpurun_out/r3d
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
STAGES="${STAGES:-tests diag noniid}"
for st in $STAGES; do
  case $st in
    tests)
      timeout -k 10 900 python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_cnn_native_gpu.py \
        tests/test_peer_comm_gpu.py -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
      echo "tests rc=$rc" >> $S; grep -E "FAILED|passed|failed" $O/tests.log | tail -12 >> $S; stop $rc
      FEDMI_FAILOVER_REPORT=$O/drills8.jsonl timeout -k 10 900 python -u -m pytest tests/test_failover_kill.py -v \
        -k "gpu" --timeout 420 --timeout-method thread > $O/drills.log 2>&1; rc=$?
      echo "drills rc=$rc" >> $S; grep -E "FAILED|passed|failed" $O/drills.log | tail -6 >> $S; stop $rc ;;
    diag)
      timeout -k 10 600 python tools/diag_engine_parity.py ResNet18 MobileNet MobileNetV2 > $O/parity.log 2>&1; rc=$?
      echo "parity rc=$rc" >> $S; cat $O/parity.log >> $S; stop $rc
      timeout -k 10 600 python tools/diag_engine_parity.py ResNet18 MobileNetV2 --warm 30 > $O/parity_warm.log 2>&1; rc=$?
      echo "parity warm rc=$rc" >> $S; cat $O/parity_warm.log >> $S; stop $rc ;;
    noniid)
      export FEDMI_BENCH_REHEARSE=1
      for split in iid noniid; do
        extra=""; [ "$split" = noniid ] && extra="--noniid 2"
        timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
          --master-port $((29500 + RANDOM % 1000)) bench.py --model resnet18 --gpus 2 --steps 7 --warmup 1 \
          --eval-full $extra --json-out $O/resnet18_2c_$split.json > $O/resnet18_2c_$split.log 2>&1; rc=$?
        echo "bench $split rc=$rc" >> $S; tail -1 $O/resnet18_2c_$split.log | cut -c1-600 >> $S; stop $rc
      done ;;
  esac
done
echo done >> $S
