set -o pipefail
mkdir -p gpurun_out
for m in resnet18 mobilenet; do
  timeout -k 10 300 python bench.py --model $m --steps 2 --warmup 1 > gpurun_out/bench_$m.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --model resnet18 --noniid 2 --steps 2 --warmup 1 > gpurun_out/bench_resnet18_noniid.log 2>&1 || exit $?
FEDMI_TORCH_PATH=1 timeout -k 10 400 python bench.py --model resnet18 --steps 1 --warmup 1 > gpurun_out/bench_resnet18_torch.log 2>&1 || exit $?
FEDMI_TORCH_PATH=1 timeout -k 10 400 python bench.py --model mobilenet --steps 1 --warmup 1 > gpurun_out/bench_mobilenet_torch.log 2>&1 || exit $?
