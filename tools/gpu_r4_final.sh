#!/bin/bash
# Round-4 final validation, part 1: the whole GPU suite.
T=${1:-r4v}
bash tools/gpu_steps.sh $T \
  gpusuite 1000 "python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
