#!/bin/bash
# full GPU validation: the GPU test suite, smoke, the 1-GPU bench
set -u
O=gpurun_out/r3full
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $O/tests.log)" >> $O/summary.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc $(tail -1 $O/smoke.log)" >> $O/summary.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc" >> $O/summary.txt; tail -1 $O/bench.log >> $O/summary.txt
