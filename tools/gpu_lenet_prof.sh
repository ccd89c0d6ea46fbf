#!/bin/bash
# LeNet step profile: kernel trace + two PMC passes + the s_memtime stamps build.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/${1:-lenet_prof}
mkdir -p $out
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python bench.py --steps 5 --warmup 2 > $out/kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $out/pmc1 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-graph > $out/pmc1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM -d $out/pmc2 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-graph > $out/pmc2.log 2>&1 || exit $?
if [ -f tools/diag_stamps.py ]; then timeout -k 10 180 python tools/diag_stamps.py > $out/stamps.txt 2>&1 || exit $?; fi
echo done > $out/done.txt
