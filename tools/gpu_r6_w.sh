# round 6: generic WGRAD split-count sweep at the GoogLeNet / DenseNet / MobileNet 1x1 and narrow shapes
bash tools/gpu_steps.sh r6_w probe 400 "python -u tools/probes/wgrad_split_probe.py"
