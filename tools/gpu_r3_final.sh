#!/bin/bash
# round-3 closing run: GPU suite + smoke + bench (gpu_r3_full.sh), then the LeNet profile reconcile
set -u
bash tools/gpu_r3_full.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_r3_reconcile.sh
