#!/bin/bash
# after replacing the graph-captured stats memset with a kernel: the system diag variants, then the system /
# LeNet GPU tests
set -u
O=gpurun_out/r3sf
mkdir -p $O
run() {  # tag, env, args...
  local tag=$1 envs=$2; shift 2
  env $envs PYTHONUNBUFFERED=1 DIAG_TAIL=20 timeout -k 10 120 python -u tools/diag_system_topk.py "$@" > $O/$tag.log 2>&1; local rc=$?
  echo "== $tag rc=$rc $(grep -c 'stats flag' $O/$tag.log) flag-failures $(grep RESULT $O/$tag.log)" >> $O/summary.txt
  return $rc
}
run y_topk "X=1" peer Y || [ $? -eq 1 ] || exit 1
run y_none_1client "DIAG_CLIENTS=1" peer Y --compress none || [ $? -eq 1 ] || exit 1
run n_none "X=1" peer N || [ $? -eq 1 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_system_gpu.py tests/test_lenet_kernels_gpu.py -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $O/tests.log)" >> $O/summary.txt
