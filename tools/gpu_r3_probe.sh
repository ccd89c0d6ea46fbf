#!/bin/bash
# -c Y system path with per-phase stats probes (client logs), then the native-mode exactness A/B.
set -u
O=gpurun_out/r3p
mkdir -p $O
FEDMI_DEBUG_STATS=1 DIAG_TAIL=150 timeout -k 10 150 python tools/diag_system_topk.py peer Y > $O/diag_probe.log 2>&1; rc=$?
echo "probe rc=$rc" > $O/summary.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_r3_exact.sh
