# round 6: weight gradients on a second graph branch (A/B), and the lr-0.1 non-IID seed gate
o=gpurun_out/r6_c
args=()
for m in resnet18 mobilenet; do
  args+=(${m}_base 200 "python bench.py --model $m --steps 3 --warmup 1 --json-out $o/${m}_base.json")
  for d in 1 2 4; do
    args+=(${m}_ws$d 200 "FEDMI_WGRAD_STREAM=1 FEDMI_WGRAD_SPLIT_DIV=$d python bench.py --model $m --steps 3 --warmup 1 --json-out $o/${m}_ws$d.json")
  done
  args+=(${m}_base2 200 "python bench.py --model $m --steps 3 --warmup 1 --json-out $o/${m}_base2.json")
done
args+=(noniid 600 "python -u -m pytest tests/test_noniid_gpu.py -k 'reference_lr or config3' -x -v -s --timeout 420 --timeout-method thread -p no:cacheprovider")
bash tools/gpu_steps.sh r6_c "${args[@]}"
