#!/bin/bash
# non-IID native-engine bench collapse: isolate the data plane (peer vs gloo) and graph replay.
set -u
O=gpurun_out/r3n
mkdir -p $O
S=$O/summary.txt
export FEDMI_BENCH_REHEARSE=1
for v in "gloo:--allreduce rccl" "nograph:--no-graph" "peer:"; do
  tag=${v%%:*}; extra=${v#*:}
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --model resnet18 --gpus 2 --steps 1 --warmup 1 \
    --eval-full --noniid 2 --trace $extra > $O/$tag.log 2>&1; rc=$?
  echo "$tag rc=$rc" >> $S; grep trace $O/$tag.log >> $S
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 300 python tools/fedavg_sim.py --model resnet18 --clients 2 --noniid 2 --rounds 2 --engine native > $O/sim.log 2>&1
echo "sim rc=$?" >> $S; cat $O/sim.log >> $S
echo done >> $S
