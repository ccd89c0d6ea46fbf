#!/bin/bash
# -c Y system path: which ingredient corrupts the LeNet train stats (compressor kind, gzip, LeNet path)
set -u
O=gpurun_out/r3sv
mkdir -p $O
run() {  # tag, env, args...
  local tag=$1 envs=$2; shift 2
  env $envs PYTHONUNBUFFERED=1 FEDMI_DEBUG_STATS=1 DIAG_TAIL=60 timeout -k 10 120 python -u tools/diag_system_topk.py "$@" > $O/$tag.log 2>&1; local rc=$?
  echo "== $tag rc=$rc $(grep -c 'stats flag' $O/$tag.log) flag-failures $(grep RESULT $O/$tag.log)" >> $O/summary.txt
  return $rc
}
run y_none "X=1" peer Y --compress none || [ $? -eq 1 ] || exit 1
run y_int8 "X=1" peer Y --compress int8 || [ $? -eq 1 ] || exit 1
run n_topk "X=1" peer N --compress topk || [ $? -eq 1 ] || exit 1
run y_topk_head "FEDMI_LENET_PATH=head" peer Y || [ $? -eq 1 ] || exit 1
echo done >> $O/summary.txt
