# round 6: attribute the lr-0.1 non-IID gap (stem kernel / WGRAD split rounding) and DPN26 at lr 0.02
bash tools/gpu_steps.sh r6_j \
  lr01_base 400 "python -u -m pytest tests/test_noniid_gpu.py -k reference_lr -q -s --timeout 380 --timeout-method thread -p no:cacheprovider" ; \
bash tools/gpu_steps.sh r6_j2 \
  lr01_nostem 400 "FEDMI_STEM=0 python -u -m pytest tests/test_noniid_gpu.py -k reference_lr -q -s --timeout 380 --timeout-method thread -p no:cacheprovider" ; \
bash tools/gpu_steps.sh r6_j3 \
  lr01_splitup 400 "FEDMI_WGRAD_SPLITS_UP=1 python -u -m pytest tests/test_noniid_gpu.py -k reference_lr -q -s --timeout 380 --timeout-method thread -p no:cacheprovider" ; \
bash tools/gpu_steps.sh r6_j4 \
  lr01_both 400 "FEDMI_STEM=0 FEDMI_WGRAD_SPLITS_UP=1 python -u -m pytest tests/test_noniid_gpu.py -k reference_lr -q -s --timeout 380 --timeout-method thread -p no:cacheprovider"
exit 0
