# round 6: 1x1 WGRAD per shape, halo<1,1> vs generic
bash tools/gpu_steps.sh r6_aq \
  on 200 "env FEDMI_WGRAD_1X1=1 python -u tools/probes/wgrad1x1_halo_probe.py" \
  off 200 "env FEDMI_WGRAD_1X1=0 python -u tools/probes/wgrad1x1_halo_probe.py"
