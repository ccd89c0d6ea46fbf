#!/bin/bash
# One GPU-box session: build check, GPU tests, smoke, bench, rocprof profile.
# Every GPU step has its own time limit; a crash-class exit (>=124 or signal)
# stops the script so nothing else touches the GPU after a fault.
set -u
mkdir -p gpurun_out
ok_or_stop() {  # $1 = exit code of a GPU step; pytest "tests failed" (1) is not a fault
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: GPU step exited $1" | tee -a gpurun_out/summary.txt; exit "$1"; fi
}
STAGES="${STAGES:-tests smoke bench prof}"
for st in $STAGES; do
  case $st in
    tests) timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/tests.log 2>&1; rc=$?
           echo "tests rc=$rc" >> gpurun_out/summary.txt; tail -5 gpurun_out/tests.log >> gpurun_out/summary.txt; ok_or_stop $rc ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
           echo "smoke rc=$rc" >> gpurun_out/summary.txt; tail -3 gpurun_out/smoke.log >> gpurun_out/summary.txt; ok_or_stop $rc ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
           echo "bench rc=$rc" >> gpurun_out/summary.txt; tail -3 gpurun_out/bench.log >> gpurun_out/summary.txt; ok_or_stop $rc ;;
    diag)  timeout -k 10 400 python tools/diag_convergence.py ${DIAG_EPOCHS:-4} > gpurun_out/diag.log 2>&1; rc=$?
           echo "diag rc=$rc" >> gpurun_out/summary.txt; tail -6 gpurun_out/diag.log >> gpurun_out/summary.txt; ok_or_stop $rc ;;
    stamps) timeout -k 10 300 env FEDMI_NATIVE_VARIANT=stamps python tools/diag_stamps.py > gpurun_out/stamps.log 2>&1; rc=$?
           echo "stamps rc=$rc" >> gpurun_out/summary.txt; cat gpurun_out/stamps.log >> gpurun_out/summary.txt; ok_or_stop $rc ;;
    prof)  (cd /tmp && export TMPDIR=/tmp && true); export TMPDIR=/tmp
           timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof.log 2>&1; rc=$?
           echo "prof rc=$rc" >> gpurun_out/summary.txt; ok_or_stop $rc ;;
  esac
done
echo done >> gpurun_out/summary.txt
