# round 6: small-layer WGRAD side stream A/B + end-of-round CNN / LeNet kernel profiles
o=gpurun_out/r6_i
mkdir -p $o
args=()
for m in mobilenet resnet18; do
  args+=(${m}_base 200 "python bench.py --model $m --steps 3 --warmup 1 --json-out $o/${m}_base.json")
  for px in 2048 8192; do
    args+=(${m}_side$px 200 "FEDMI_WGRAD_SIDE_MAXPIX=$px python bench.py --model $m --steps 3 --warmup 1 --json-out $o/${m}_side$px.json")
  done
  args+=(${m}_base2 200 "python bench.py --model $m --steps 3 --warmup 1 --json-out $o/${m}_base2.json")
done
args+=(prof 600 "MODELS='resnet18 mobilenet lenet' bash tools/gpu_prof_models.sh r6_i/prof")
bash tools/gpu_steps.sh r6_i "${args[@]}"
