#!/bin/bash
# Round-4: where the N=8 projection's wall time goes beyond the device span -- the checkpoint writer.
# Interleaved: default (4 slots, every round written), 16 slots, coalescing, /dev/shm target.
T=${1:-r4k}
p="python bench.py --breakdown --project-world 8 --steps 60 --warmup 5"
bash tools/gpu_steps.sh $T \
  def1 90 "$p --json-out gpurun_out/$T/def1.json" \
  s16_1 90 "$p --ckpt-slots 16 --json-out gpurun_out/$T/s16_1.json" \
  coal1 90 "$p --ckpt-coalesce --json-out gpurun_out/$T/coal1.json" \
  shm1 90 "$p --ckpt-dir /dev/shm/fedmi_ck_$$ --json-out gpurun_out/$T/shm1.json" \
  def2 90 "$p --json-out gpurun_out/$T/def2.json" \
  s16_2 90 "$p --ckpt-slots 16 --json-out gpurun_out/$T/s16_2.json" \
  coal2 90 "$p --ckpt-coalesce --json-out gpurun_out/$T/coal2.json" \
  shm2 90 "$p --ckpt-dir /dev/shm/fedmi_ck_$$ --json-out gpurun_out/$T/shm2.json"
rm -rf /dev/shm/fedmi_ck_$$
