# round 6: one checkpoint write of the LeNet state, device idle (the timed-region tail of bench.py)
bash tools/gpu_steps.sh r6_ad probe 200 "python -u tools/probes/ckpt_write_probe.py"
