#!/bin/bash
# -c Y system path, round 2: graph vs eager LeNet, one client vs two, dense no-gzip with probes
set -u
O=gpurun_out/r3sv2
mkdir -p $O
run() {  # tag, env, args...
  local tag=$1 envs=$2; shift 2
  env $envs PYTHONUNBUFFERED=1 FEDMI_DEBUG_STATS=1 DIAG_TAIL=60 timeout -k 10 120 python -u tools/diag_system_topk.py "$@" > $O/$tag.log 2>&1; local rc=$?
  echo "== $tag rc=$rc $(grep -c 'stats flag' $O/$tag.log) flag-failures $(grep RESULT $O/$tag.log)" >> $O/summary.txt
  return $rc
}
run n_none "X=1" peer N || [ $? -eq 1 ] || exit 1
run y_none_eager "X=1" peer Y --compress none --no-graph || [ $? -eq 1 ] || exit 1
run y_none_1client "DIAG_CLIENTS=1" peer Y --compress none || [ $? -eq 1 ] || exit 1
run y_none_3client "DIAG_CLIENTS=3" peer Y --compress none || [ $? -eq 1 ] || exit 1
echo done >> $O/summary.txt
