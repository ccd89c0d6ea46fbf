#!/bin/bash
# Round-4: every zoo family on the native aten backend against PyTorch fp32, one box, one call.
T=${1:-r4za}
bash tools/gpu_steps.sh $T \
  zooall 900 "BENCH_MODES=fp32,native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 ResNeXt29_2x64d ResNeXt29_32x4d DPN26 DPN92 ShuffleNetG2 ShuffleNetG3 ShuffleNetV2 SENet18 EfficientNetB0 RegNetX_200MF RegNetY_400MF PNASNetA PNASNetB DLA SimpleDLA > gpurun_out/$T/zoo_all.jsonl"
