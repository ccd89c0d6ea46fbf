# round 6: re-run the three suite failures (DPN26 at lr 0.005, 5-seed lr-0.1 gate, config-3 peak on the seed mean)
bash tools/gpu_steps.sh r6_k \
  fixes 900 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_noniid_gpu.py -k 'family or reference_lr or config3' -q -s --timeout 600 --timeout-method thread -p no:cacheprovider"
