#!/bin/bash
# Three rocprofv3 PMC passes (SQ counters only, each pass within the per-block slot limits, each under its
# own hard time limit) over one command; CSV output under gpurun_out/<tag>/pmc{1,2,3}.
#   usage: bash tools/gpu_pmc.sh <tag> <command...>
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM"
P3="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for p in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $p -d "$out/pmc$i" -o run --output-format csv -- "$@" > "$out/pmc$i.log" 2>&1
  rc=$?
  echo "pmc$i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
