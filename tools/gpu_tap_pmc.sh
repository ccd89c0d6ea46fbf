#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_tap.py --iters 30 > gpurun_out/bench_tap.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d gpurun_out/pmc1 -o run --output-format csv -- python tools/bench_tap.py --iters 3 --shapes l1,l4 > gpurun_out/pmc1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM -d gpurun_out/pmc2 -o run --output-format csv -- python tools/bench_tap.py --iters 3 --shapes l1,l4 > gpurun_out/pmc2.log 2>&1 || exit $?
echo done > gpurun_out/pmc_done.txt
