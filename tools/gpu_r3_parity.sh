#!/bin/bash
# Round 3: non-IID parity (native vs fp32 PyTorch, in-process FedAvg simulator), the 8-client
# failover drills (config 5), and the product path re-measured at HEAD (bench_system.py).
set -u
O=gpurun_out/r3p
mkdir -p $O
S=$O/summary.txt
stop() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: step exited $1" | tee -a $S; exit "$1"; fi; }
STAGES="${STAGES:-sim drills sys}"
for st in $STAGES; do
  case $st in
    sim)
      for eng in native fp32; do
        timeout -k 10 300 python tools/fedavg_sim.py --model resnet18 --clients 2 --noniid 2 --rounds 8 --engine $eng \
          --out $O/noniid_$eng.jsonl > $O/sim_noniid_$eng.log 2>&1; rc=$?
        echo "sim noniid $eng rc=$rc" >> $S; tail -1 $O/sim_noniid_$eng.log >> $S; stop $rc
        timeout -k 10 300 python tools/fedavg_sim.py --model resnet18 --clients 2 --rounds 4 --engine $eng \
          --out $O/iid_$eng.jsonl > $O/sim_iid_$eng.log 2>&1; rc=$?
        echo "sim iid $eng rc=$rc" >> $S; tail -1 $O/sim_iid_$eng.log >> $S; stop $rc
      done ;;
    drills)
      FEDMI_FAILOVER_REPORT=$O/drills8.jsonl timeout -k 10 900 python -u -m pytest tests/test_failover_kill.py -x -v \
        -k "8_clients_gpu" --timeout 420 --timeout-method thread > $O/drills.log 2>&1; rc=$?
      echo "drills rc=$rc" >> $S; tail -3 $O/drills.log >> $S; stop $rc ;;
    sys)
      for n in 1 2; do
        timeout -k 10 400 python bench_system.py --clients $n --rounds 30 --warmup 5 --json-out $O/sys_lenet_$n.json \
          > $O/sys_lenet_$n.log 2>&1; rc=$?
        echo "sys lenet $n rc=$rc" >> $S; tail -1 $O/sys_lenet_$n.log >> $S; stop $rc
      done
      timeout -k 10 500 python bench_system.py --model mobilenet --clients 2 --rounds 6 --warmup 2 \
        --json-out $O/sys_mobilenet_2.json > $O/sys_mobilenet_2.log 2>&1; rc=$?
      echo "sys mobilenet 2 rc=$rc" >> $S; tail -1 $O/sys_mobilenet_2.log >> $S; stop $rc ;;
  esac
done
echo done >> $S
