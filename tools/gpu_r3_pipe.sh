#!/bin/bash
# LeNet pipelined epoch (SGD(i-1) + samples(i) per launch): bit-identity tests, then A/B bench runs.
set -u
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lenet_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "pipelined or graph_epoch or sample_path or sgd_kernel" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2 3; do
  for pipe in 0 1; do
    FEDMI_LENET_PIPE=$pipe timeout -k 10 240 python bench.py --json-out $O/bench_pipe${pipe}_$i.json > $O/bench_pipe${pipe}_$i.log 2>&1 || exit $?
    echo "pipe=$pipe run=$i $(python -c "import json;d=json.load(open('$O/bench_pipe${pipe}_$i.json'));print(d['value'], d['ms_per_step'])")"
  done
done
echo done
