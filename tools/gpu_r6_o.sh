# round 6: GoogLeNet deferred-WGRAD mismatch -- per-conv probe
bash tools/gpu_steps.sh r6_o \
  probe 300 "python -u tools/probes/wred_defer_probe.py GoogLeNet" \
  probe_r18 300 "python -u tools/probes/wred_defer_probe.py ResNet18"
