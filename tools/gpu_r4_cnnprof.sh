#!/bin/bash
# Round-4: per-kernel time of one ResNet-18 and one MobileNet bench configuration (kernel trace + stats).
T=${1:-r4cp}
export TMPDIR=/tmp
bash tools/gpu_steps.sh $T \
  r18prof 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/$T/r18 -o p --output-format csv -- python bench.py --model resnet18 --steps 2 --warmup 1 --json-out gpurun_out/$T/r18.json" \
  mbnprof 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/$T/mbn -o p --output-format csv -- python bench.py --model mobilenet --steps 2 --warmup 1 --json-out gpurun_out/$T/mbn.json"
# keep the per-kernel summaries only (the full traces exceed the 64 MiB gpurun_out cap)
python tools/trace_top.py gpurun_out/$T/r18/p_kernel_trace.csv > gpurun_out/$T/r18_top.txt 2>&1
python tools/trace_top.py gpurun_out/$T/mbn/p_kernel_trace.csv > gpurun_out/$T/mbn_top.txt 2>&1
rm -f gpurun_out/$T/*/p_kernel_trace.csv
exit 0
