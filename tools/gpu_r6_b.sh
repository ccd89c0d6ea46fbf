# round 6: re-landed CNN wins + multi-seed parity gates + kernel lists + peer abort word
bash tools/gpu_steps.sh r6_b \
  kern 400 "python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_kernel_list_gpu.py tests/test_peer_comm_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  bench 150 "python bench.py --json-out gpurun_out/r6_b/bench1.json" \
  r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/r6_b/r18.json" \
  mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/r6_b/mbn.json" \
  family 500 "python -u -m pytest tests/test_native_mode_gpu.py -k family -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider" \
  noniid 900 "python -u -m pytest tests/test_noniid_gpu.py -x -v -s --timeout 420 --timeout-method thread -p no:cacheprovider"
