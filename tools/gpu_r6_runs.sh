#!/bin/bash
# Round-6 GPU runs behind profiles/r6_* (one arm per experiment; each arm's first comment names it).
#   usage: bash tools/gpu_r6_runs.sh <run>        e.g.  bash tools/gpu_r6_runs.sh at
#   list:  bash tools/gpu_r6_runs.sh list
# Every arm drives tools/gpu_steps.sh (named steps, each under its own time limit; the first failing step ends
# the run).  Outputs land in gpurun_out/r6_<run>/.  The whole GPU suite + smoke is tools/gpu_r6_suite.sh.
run=${1:?run name, or "list"}; shift
case "$run" in
  a)
    # round 6: first CNN / LeNet measurements at the round-5 HEAD
    bash tools/gpu_steps.sh r6_a \
      bench 150 "python bench.py --json-out gpurun_out/r6_a/bench1.json" \
      r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/r6_a/r18.json" \
      mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/r6_a/mbn.json" \
      failover 600 "FEDMI_FAILOVER_REPORT=gpurun_out/r6_a/drills.jsonl python -u -m pytest tests/test_failover_kill.py -k 'client_sigkill and gpu' -x -v --timeout 420 --timeout-method thread -p no:cacheprovider"
    ;;
  aa)
    # round 6: LeNet eval conv forward at 6 waves / SIMD (three workgroups per CU) -- tests + breakdown + stats
    set -e
    export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
    out=gpurun_out/${TAG:-r6_aa}
    mkdir -p $out
    timeout -k 10 300 python3 -u -m pytest tests/test_lenet_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
    tail -n 2 $out/tests.log
    timeout -k 10 300 python3 bench.py --breakdown > $out/lenet_breakdown.log 2>&1
    timeout -k 10 300 python3 bench.py > $out/lenet2.log 2>&1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/lenet -o run -- python3 bench.py --steps 3 --warmup 1 > $out/lenet_prof.log 2>&1
    st=$(find $out/lenet -name 'run_kernel_stats.csv' | head -n 1)
    python3 tools/prof_summary.py "$st" lenet_sgd2 30 > $out/lenet_kernels.txt
    rm -f $(find $out/lenet -name 'run_kernel_trace.csv')
    grep "onv_fwd\|fc_eval" $out/lenet_kernels.txt || true
    ;;
  ac)
    # round 6: product-path refresh (bench_system.py: server.py primary + backup + client.py processes over gRPC)
    bash tools/gpu_steps.sh r6_ac \
      lenet1 300 "python -u bench_system.py --clients 1 --rounds 60 --warmup 10 --json-out gpurun_out/r6_ac/lenet1.json" \
      lenet2 300 "python -u bench_system.py --clients 2 --rounds 60 --warmup 10 --json-out gpurun_out/r6_ac/lenet2.json" \
      mbn2 400 "python -u bench_system.py --clients 2 --model mobilenet --rounds 10 --warmup 3 --json-out gpurun_out/r6_ac/mbn2.json"
    ;;
  ad)
    # round 6: one checkpoint write of the LeNet state, device idle (the timed-region tail of bench.py)
    bash tools/gpu_steps.sh r6_ad probe 200 "python -u tools/probes/ckpt_write_probe.py"
    ;;
  ae)
    # round 6: LeNet per-round device spans (where the mean round exceeds the median)
    bash tools/gpu_steps.sh r6_ae \
      b1 200 "python -u bench.py --breakdown --steps 40 --warmup 3" \
      b2 200 "python -u bench.py --breakdown --steps 40 --warmup 3"
    ;;
  af)
    # round 6: LeNet slow rounds 2-4 of the timed region -- vary the checkpoint writer's slots and the warmup
    bash tools/gpu_steps.sh r6_af \
      s1 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 1" \
      s2 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 2" \
      s16 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 16" \
      w10 200 "python -u bench.py --breakdown --steps 30 --warmup 10" \
      noev 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --no-eval"
    ;;
  ag)
    # round 6: checkpoint writer slots touched at construction -- the slow rounds 2-4 should be gone
    bash tools/gpu_steps.sh r6_ag \
      d4 200 "python -u bench.py --breakdown --steps 30 --warmup 3" \
      s16 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 16" \
      def 200 "python -u bench.py" \
      def2 200 "python -u bench.py"
    ;;
  ah)
    # round 6: bench.py with the 2-slot checkpoint writer default
    bash tools/gpu_steps.sh r6_ah \
      def 200 "python -u bench.py" \
      def2 200 "python -u bench.py" \
      w1 200 "python -u bench.py --warmup 1 --steps 20 --breakdown" \
      k50 200 "python -u bench.py --warmup 2 --steps 50 --breakdown"
    ;;
  ai)
    # round 6: LeNet epoch graph double-instanced (alternate launches) -- slow-round check at 4 / 16 slots and default
    bash tools/gpu_steps.sh r6_ai \
      s4 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 4" \
      s16 200 "python -u bench.py --breakdown --steps 30 --warmup 3 --ckpt-slots 16" \
      w1 200 "python -u bench.py --warmup 1 --steps 20 --breakdown" \
      def 200 "python -u bench.py"
    ;;
  aj)
    # round 6: CNN benches with the 2-slot checkpoint writer default (vs 4)
    bash tools/gpu_steps.sh r6_aj \
      r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1 --breakdown" \
      r18_s4 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1 --ckpt-slots 4 --breakdown" \
      mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1 --breakdown" \
      mbn_s4 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1 --ckpt-slots 4 --breakdown"
    ;;
  ak)
    # round 6: N=8 per-client projection (1 GPU, rank 0's shard, full eval) with the round breakdown
    bash tools/gpu_steps.sh r6_ak \
      p8 200 "python -u bench.py --project-world 8 --steps 100 --warmup 5 --breakdown" \
      p8b 200 "python -u bench.py --project-world 8 --steps 100 --warmup 5"
    ;;
  al)
    # round 6: split-K FWD/DGRAD combine with 2 splits' loads in flight per step (bit-identical) -- tests + A/B
    bash tools/gpu_steps.sh r6_al \
      kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'conv or fused or tap'" \
      r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      r18b 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
      mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
    ;;
  am)
    # round 6: BN-backward reduce with two rows' loads in flight (bit-identical) -- tests + A/B
    bash tools/gpu_steps.sh r6_am \
      kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'bn'" \
      eng 300 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'deterministic'" \
      goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
      mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      goog2 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
      mbn2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
    ;;
  an)
    # round 6: split-K combine with 4 splits' loads in flight per step (vs 2) -- tests + A/B
    bash tools/gpu_steps.sh r6_an \
      kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'conv or fused or tap'" \
      r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      r18b 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
      mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
    ;;
  ao)
    # round 6: final N>1 rehearsal of bench.py on one GPU (ranks time-slice the card; peer transport verified vs gloo)
    o=gpurun_out/r6_ao
    mkdir -p $o
    bash tools/gpu_steps.sh r6_ao \
      reh2 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 5 --warmup 2 --json-out $o/reh2.json" \
      reh4 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 4 --steps 5 --warmup 2 --json-out $o/reh4.json"
    ;;
  ap)
    # round 6: 1x1 WGRAD on conv_wgrad_halo<1, 1> -- kernel tests, engine bit-identity tests, A/B (FEDMI_WGRAD_1X1=0)
    bash tools/gpu_steps.sh r6_ap \
      kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'wgrad or dgrad'" \
      eng 300 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'deterministic or deferred'" \
      mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      mbn_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
      goog_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model googlenet --steps 2 --warmup 1" \
      r18 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      mbn2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
    ;;
  aq)
    # round 6: 1x1 WGRAD per shape, halo<1,1> vs generic
    bash tools/gpu_steps.sh r6_aq \
      on 200 "env FEDMI_WGRAD_1X1=1 python -u tools/probes/wgrad1x1_halo_probe.py" \
      off 200 "env FEDMI_WGRAD_1X1=0 python -u tools/probes/wgrad1x1_halo_probe.py"
    ;;
  ar)
    # round 6: 1x1 halo WGRAD limited to small problems -- tests + A/B
    bash tools/gpu_steps.sh r6_ar \
      kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'wgrad'" \
      eng 300 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'deterministic or deferred'" \
      mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      goog 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
      goog_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model googlenet --steps 2 --warmup 1" \
      mbn2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      mbn_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model mobilenet --steps 3 --warmup 1"
    ;;
  as)
    # round 6: 1x1 halo WGRAD A/B beyond MobileNet -- MobileNetV2 (CNN engine) and the aten-backend zoo
    M="densenet_cifar DenseNet121 DPN26 RegNetX_200MF RegNetY_400MF SimpleDLA EfficientNetB0 ResNeXt29_2x64d SENet18"
    bash tools/gpu_steps.sh r6_as \
      mbv2 300 "python -u bench.py --model mobilenetv2 --steps 2 --warmup 1" \
      mbv2_off 300 "env FEDMI_WGRAD_1X1=0 python -u bench.py --model mobilenetv2 --steps 2 --warmup 1" \
      zoo 400 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M" \
      zoo_off 400 "env BENCH_MODES=native-graph FEDMI_WGRAD_1X1=0 python -u tools/bench_hybrid.py $M"
    ;;
  at)
    # round 6: 1x1 halo WGRAD kept to the CNN engine (aten backend: generic) -- tests + zoo / MobileNet check
    M="densenet_cifar DPN26 SENet18 ResNeXt29_2x64d"
    bash tools/gpu_steps.sh r6_at \
      kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'wgrad'" \
      zoot 400 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_kernel_list_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'deferred or launches or conv_fwd_bwd'" \
      mbn 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      zoo 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M"
    ;;
  b)
    # round 6: re-landed CNN wins + multi-seed parity gates + kernel lists + peer abort word
    bash tools/gpu_steps.sh r6_b \
      kern 400 "python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_kernel_list_gpu.py tests/test_peer_comm_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
      bench 150 "python bench.py --json-out gpurun_out/r6_b/bench1.json" \
      r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/r6_b/r18.json" \
      mbn 200 "python bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/r6_b/mbn.json" \
      family 500 "python -u -m pytest tests/test_native_mode_gpu.py -k family -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider" \
      noniid 900 "python -u -m pytest tests/test_noniid_gpu.py -x -v -s --timeout 420 --timeout-method thread -p no:cacheprovider"
    ;;
  c)
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
    ;;
  cd)
    # round 6: first CNN / LeNet measurements at the round-5 HEAD
    bash "$0" d && bash "$0" c
    ;;
  d)
    # round 6: fused -c Y int8 peer collective (test + timing), N>1 bench rehearsal with the split-eval compare loop,
    # GoogLeNet kernel breakdown
    o=gpurun_out/r6_d
    mkdir -p $o
    export HSA_ENABLE_IPC_MODE_LEGACY=0
    bash tools/gpu_steps.sh r6_d \
      int8test 300 "python -u -m pytest tests/test_peer_comm_gpu.py -k 'int8 or abort' -x -v --timeout 240 --timeout-method thread -p no:cacheprovider" \
      peerbench 300 "python tools/bench_peer.py --world 2 4 --iters 200 --no-gate --out $o/peer_nogate.jsonl" \
      reh2 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --json-out $o/reh2.json" \
      reh4y 300 "FEDMI_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 5 --warmup 2 --compress Y --json-out $o/reh4y.json" \
      googprof 300 "MODELS=googlenet bash tools/gpu_prof_models.sh r6_d/prof"
    ;;
  e)
    # round 6: KS2 SGD operands loaded first (LeNet), then the c+d batch
    bash tools/gpu_steps.sh r6_e \
      lenettest 300 "python -u -m pytest tests/test_lenet_kernels_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
      bench_a 150 "python bench.py --json-out gpurun_out/r6_e/bench_a.json" \
      bench_b 150 "python bench.py --json-out gpurun_out/r6_e/bench_b.json" && bash "$0" d && bash "$0" c
    ;;
  f)
    # round 6: GEN conv_tap forward (C % 8), vectorised fused int8 peer collective
    o=gpurun_out/r6_f
    mkdir -p $o
    export HSA_ENABLE_IPC_MODE_LEGACY=0
    bash tools/gpu_steps.sh r6_f \
      kern 400 "python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_peer_comm_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
      zoo 600 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_cnn_native_gpu.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider" \
      peerbench 300 "python tools/bench_peer.py --world 2 4 --iters 200 --no-gate --out $o/peer_nogate.jsonl" \
      goog 300 "python bench.py --model googlenet --steps 2 --warmup 1 --json-out $o/goog.json" \
      r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out $o/r18.json" \
      zoobench 400 "BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 DLA DPN26 PNASNetA > $o/zoo.jsonl" \
      googprof 300 "MODELS=googlenet bash tools/gpu_prof_models.sh r6_f/prof"
    ;;
  g)
    # round 6: GEN conv_tap A/B on the zoo trajectories, blocked maxpool3, fused int8 timing, GoogLeNet
    o=gpurun_out/r6_g
    mkdir -p $o
    export HSA_ENABLE_IPC_MODE_LEGACY=0
    bash tools/gpu_steps.sh r6_g \
      kern 400 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
      dpn_gen0 300 "FEDMI_TAP_GEN=0 python -u -m pytest tests/test_native_mode_gpu.py -k 'family and DPN26' -x -q -s --timeout 280 --timeout-method thread -p no:cacheprovider" \
      dpn_gen1 300 "python -u -m pytest tests/test_native_mode_gpu.py -k 'family and DPN26' -x -q -s --timeout 280 --timeout-method thread -p no:cacheprovider" \
      zoo 600 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_cnn_native_gpu.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider" \
      peerbench 300 "python tools/bench_peer.py --world 2 4 --iters 200 --no-gate --out $o/peer_nogate.jsonl" \
      goog 300 "python bench.py --model googlenet --steps 2 --warmup 1 --json-out $o/goog.json" \
      goog_gen0 300 "FEDMI_TAP_GEN=0 python bench.py --model googlenet --steps 2 --warmup 1 --json-out $o/goog_gen0.json" \
      r18 200 "python bench.py --model resnet18 --steps 3 --warmup 1 --json-out $o/r18.json" \
      zoobench 400 "BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 DLA DPN26 PNASNetA > $o/zoo.jsonl" \
      zoobench0 400 "FEDMI_TAP_GEN=0 BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 DLA DPN26 PNASNetA > $o/zoo_gen0.jsonl" \
      googprof 300 "MODELS=googlenet bash tools/gpu_prof_models.sh r6_g/prof"
    ;;
  h)
    # round 6: GEN conv_tap correctness sweep + zoo A/B (FEDMI_TAP_GEN=0 vs default), GoogLeNet A/B, int8 timing
    o=gpurun_out/r6_h
    mkdir -p $o
    export HSA_ENABLE_IPC_MODE_LEGACY=0
    bash tools/gpu_steps.sh r6_h \
      sweep 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -k 'gen_sweep or maxpool3' -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
      zoobench 400 "BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 DLA DPN26 PNASNetA > $o/zoo.jsonl" \
      zoobench0 400 "FEDMI_TAP_GEN=0 BENCH_MODES=native-graph python tools/bench_hybrid.py densenet_cifar DenseNet121 DLA DPN26 PNASNetA > $o/zoo_gen0.jsonl" \
      goog 300 "python bench.py --model googlenet --steps 2 --warmup 1 --json-out $o/goog.json" \
      goog_gen0 300 "FEDMI_TAP_GEN=0 python bench.py --model googlenet --steps 2 --warmup 1 --json-out $o/goog_gen0.json" \
      peerbench 300 "python tools/bench_peer.py --world 2 4 --iters 200 --no-gate --out $o/peer_nogate.jsonl" \
      fam_gen0 400 "FEDMI_TAP_GEN=0 python -u -m pytest tests/test_native_mode_gpu.py -k 'family' -q -s --timeout 380 --timeout-method thread -p no:cacheprovider" \
      fam_gen1 400 "python -u -m pytest tests/test_native_mode_gpu.py -k 'family' -q -s --timeout 380 --timeout-method thread -p no:cacheprovider"
    ;;
  i)
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
    ;;
  j)
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
    ;;
  k)
    # round 6: re-run the three suite failures (DPN26 at lr 0.005, 5-seed lr-0.1 gate, config-3 peak on the seed mean)
    bash tools/gpu_steps.sh r6_k \
      fixes 900 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_noniid_gpu.py -k 'family or reference_lr or config3' -q -s --timeout 600 --timeout-method thread -p no:cacheprovider"
    ;;
  m)
    # round 6: 1x1 WGRAD library route at <= 2048 pixels -- kernel test, MobileNet A/B (route on / off / on)
    bash tools/gpu_steps.sh r6_m \
      test 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -k 'wgrad' -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
      mbn_on 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      mbn_off 300 "env FEDMI_WGRAD_GEMM=0 python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      mbn_on2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1"
    ;;
  n)
    # round 6: deferred WGRAD reductions (one wgrad_reduce_multi launch per step) -- bit-identity, kernel list, kernel
    # tests, MobileNet / ResNet-18 A/B (FEDMI_WRED_DEFER=0 = per-conv reductions)
    bash tools/gpu_steps.sh r6_n \
      tests 600 "python -u -m pytest tests/test_cnn_native_gpu.py tests/test_kernel_list_gpu.py tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --deselect tests/test_cnn_native_gpu.py::test_loss_and_tail_grads_match_torch --deselect tests/test_cnn_native_gpu.py::test_engine_is_deterministic" \
      mbn_on 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1 --breakdown" \
      mbn_off 300 "env FEDMI_WRED_DEFER=0 python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      r18_on 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1 --breakdown" \
      r18_off 300 "env FEDMI_WRED_DEFER=0 python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      mbn_on2 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      r18_on2 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1"
    ;;
  o)
    # round 6: GoogLeNet deferred-WGRAD mismatch -- per-conv probe
    bash tools/gpu_steps.sh r6_o \
      probe 300 "python -u tools/probes/wred_defer_probe.py GoogLeNet" \
      probe_r18 300 "python -u tools/probes/wred_defer_probe.py ResNet18"
    ;;
  p)
    # round 6: HEAD kernel breakdowns after the deferred WGRAD reductions (MobileNet, ResNet-18)
    set -e
    export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
    out=gpurun_out/r6_p
    mkdir -p $out
    for m in mobilenet resnet18; do
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$m -o run -- python3 bench.py --model $m --steps 1 --warmup 1 > $out/${m}_bench.log 2>&1
      tr=$(find $out/$m -name 'run_kernel_trace.csv' | head -n 1)
      st=$(find $out/$m -name 'run_kernel_stats.csv' | head -n 1)
      python3 tools/prof_summary.py "$st" sched_next 40 > $out/${m}_kernels.txt
      python3 tools/prof_step.py "$tr" 300 > $out/${m}_step.txt
      rm -f "$tr"
      tail -n 2 $out/${m}_step.txt
    done
    ;;
  q)
    # round 6: GoogLeNet bench + kernel breakdown at HEAD (after the deferred WGRAD reductions)
    set -e
    export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
    out=gpurun_out/r6_q
    mkdir -p $out
    timeout -k 10 300 python3 bench.py --model googlenet --steps 2 --warmup 1 > $out/googlenet_bench.log 2>&1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/googlenet -o run -- python3 bench.py --model googlenet --steps 1 --warmup 1 > $out/googlenet_prof.log 2>&1
    tr=$(find $out/googlenet -name 'run_kernel_trace.csv' | head -n 1)
    st=$(find $out/googlenet -name 'run_kernel_stats.csv' | head -n 1)
    python3 tools/prof_summary.py "$st" sched_next 50 > $out/googlenet_kernels.txt
    python3 tools/prof_step.py "$tr" 300 > $out/googlenet_step.txt
    rm -f "$tr"
    tail -n 2 $out/googlenet_step.txt
    ;;
  r)
    # round 6: stride-1 DGRAD on conv_tap<GEN> (O % 8 from 16 channels) -- kernel tests, GoogLeNet engine tests, GoogLeNet A/B
    bash tools/gpu_steps.sh r6_r \
      kern 400 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
      eng 400 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'GoogLeNet or deferred'" \
      goog_on 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
      goog_off 300 "env FEDMI_TAP_GEN=0 python -u bench.py --model googlenet --steps 2 --warmup 1" \
      zoo 500 "python -u -m pytest tests/test_native_mode_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'not family'"
    ;;
  s)
    # round 6: LeNet headline at HEAD (x2) + GoogLeNet kernel breakdown after the GEN DGRAD
    set -e
    export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
    out=gpurun_out/r6_s
    mkdir -p $out
    timeout -k 10 300 python3 bench.py > $out/lenet1.log 2>&1
    timeout -k 10 300 python3 bench.py > $out/lenet2.log 2>&1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/googlenet -o run -- python3 bench.py --model googlenet --steps 1 --warmup 1 > $out/googlenet_prof.log 2>&1
    tr=$(find $out/googlenet -name 'run_kernel_trace.csv' | head -n 1)
    st=$(find $out/googlenet -name 'run_kernel_stats.csv' | head -n 1)
    python3 tools/prof_summary.py "$st" sched_next 50 > $out/googlenet_kernels.txt
    python3 tools/prof_step.py "$tr" 300 > $out/googlenet_step.txt
    rm -f "$tr"
    tail -n 1 $out/googlenet_step.txt
    ;;
  t)
    # round 6: deferred WGRAD reductions in the aten (zoo) backend -- bit-identity, kernel list, zoo A/B
    bash tools/gpu_steps.sh r6_t \
      tests 600 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_kernel_list_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'deferred or launches or graph_replay or deterministic or fusion'" \
      zoo_on 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py densenet_cifar RegNetY_400MF DLA EfficientNetB0" \
      zoo_off 300 "env BENCH_MODES=native-graph FEDMI_WRED_DEFER=0 python -u tools/bench_hybrid.py densenet_cifar RegNetY_400MF DLA EfficientNetB0"
    ;;
  u)
    # round 6: zoo A/B of the round-6 routing changes (GEN DGRAD, library 1x1 WGRAD) on the aten backend
    M="densenet_cifar DenseNet121 DPN26 RegNetX_200MF SimpleDLA"
    bash tools/gpu_steps.sh r6_u \
      base 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M" \
      nodgen 300 "env BENCH_MODES=native-graph FEDMI_DGRAD_GEN=0 python -u tools/bench_hybrid.py $M" \
      nolib 300 "env BENCH_MODES=native-graph FEDMI_WGRAD_GEMM=0 python -u tools/bench_hybrid.py $M" \
      base2 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M"
    ;;
  v)
    # round 6: zoo after restricting the GEN DGRAD / library WGRAD routes to the CNN engine; deferral on / off
    M="densenet_cifar DenseNet121 DPN26 RegNetX_200MF SimpleDLA RegNetY_400MF EfficientNetB0"
    bash tools/gpu_steps.sh r6_v \
      tests 600 "python -u -m pytest tests/test_native_mode_gpu.py tests/test_kernel_list_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'deferred or launches or graph_replay or deterministic or fusion or conv_fwd_bwd'" \
      on 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M" \
      off 300 "env BENCH_MODES=native-graph FEDMI_WRED_DEFER=0 python -u tools/bench_hybrid.py $M" \
      on2 300 "env BENCH_MODES=native-graph python -u tools/bench_hybrid.py $M"
    ;;
  w)
    # round 6: generic WGRAD split-count sweep at the GoogLeNet / DenseNet / MobileNet 1x1 and narrow shapes
    bash tools/gpu_steps.sh r6_w probe 400 "python -u tools/probes/wgrad_split_probe.py"
    ;;
  x)
    # round 6: config-3 gate after the one-sided change + smoke
    bash tools/gpu_steps.sh r6_x \
      config3 400 "python -u -m pytest tests/test_noniid_gpu.py -x -q -s --timeout 380 --timeout-method thread -p no:cacheprovider -k config3" \
      smoke 120 "python -c 'import __graft_entry__ as g; g.smoke()'" && \
    bash tools/gpu_steps.sh r6_x2 \
      vgg 300 "python -u bench.py --model vgg16 --steps 3 --warmup 1" \
      preact 300 "python -u bench.py --model preactresnet18 --steps 3 --warmup 1" \
      mbv2 300 "python -u bench.py --model mobilenetv2 --steps 3 --warmup 1"
    ;;
  y)
    # round 6: defer only small WGRAD partial sets (FEDMI_WRED_DEFER_MB), reversed reduce order -- A/B + bit-identity
    bash tools/gpu_steps.sh r6_y \
      test 400 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k deferred" \
      r18_8 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      r18_all 300 "env FEDMI_WRED_DEFER_MB=100000 python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      r18_64 300 "env FEDMI_WRED_DEFER_MB=64 python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      mbn_8 300 "python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      mbn_all 300 "env FEDMI_WRED_DEFER_MB=100000 python -u bench.py --model mobilenet --steps 3 --warmup 1" \
      r18_8b 300 "python -u bench.py --model resnet18 --steps 3 --warmup 1" \
      goog_8 300 "python -u bench.py --model googlenet --steps 2 --warmup 1" \
      goog_all 300 "env FEDMI_WRED_DEFER_MB=100000 python -u bench.py --model googlenet --steps 2 --warmup 1"
    ;;
  z)
    # round 6: LeNet round breakdown (eval share) + kernel stats of the eval path
    set -e
    export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
    out=gpurun_out/r6_z
    mkdir -p $out
    timeout -k 10 300 python3 bench.py --breakdown > $out/lenet_breakdown.log 2>&1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/lenet -o run -- python3 bench.py --steps 3 --warmup 1 > $out/lenet_prof.log 2>&1
    st=$(find $out/lenet -name 'run_kernel_stats.csv' | head -n 1)
    python3 tools/prof_summary.py "$st" lenet_sgd2 30 > $out/lenet_kernels.txt
    rm -f $(find $out/lenet -name 'run_kernel_trace.csv')
    cat $out/lenet_kernels.txt | head -20
    ;;
  final)
    # round 6: headline + CNN benches at the final HEAD (LeNet x2, ResNet-18, MobileNet, MobileNetV2, GoogLeNet)
    bash tools/gpu_steps.sh r6_final \
      lenet1 200 "python -u bench.py --json-out gpurun_out/r6_final/lenet1.json" \
      lenet2 200 "python -u bench.py --json-out gpurun_out/r6_final/lenet2.json" \
      r18 200 "python -u bench.py --model resnet18 --steps 3 --warmup 1 --json-out gpurun_out/r6_final/resnet18.json" \
      mbn 200 "python -u bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/r6_final/mobilenet.json" \
      mbv2 200 "python -u bench.py --model mobilenetv2 --steps 3 --warmup 1 --json-out gpurun_out/r6_final/mobilenetv2.json" \
      goog 250 "python -u bench.py --model googlenet --steps 3 --warmup 1 --json-out gpurun_out/r6_final/googlenet.json"
    ;;
  kfinal)
    # round 6: kernel breakdowns at the final HEAD (MobileNet / MobileNetV2 with the 1x1 halo WGRAD, ResNet-18)
    set -e
    export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
    out=gpurun_out/r6_kfinal
    mkdir -p $out
    for m in mobilenet mobilenetv2 resnet18; do
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$m -o run -- python3 bench.py --model $m --steps 1 --warmup 1 > $out/${m}_bench.log 2>&1
      tr=$(find $out/$m -name 'run_kernel_trace.csv' | head -n 1)
      st=$(find $out/$m -name 'run_kernel_stats.csv' | head -n 1)
      python3 tools/prof_summary.py "$st" sched_next 40 > $out/${m}_kernels.txt
      python3 tools/prof_step.py "$tr" 300 > $out/${m}_step.txt
      rm -f "$tr"
      tail -n 2 $out/${m}_step.txt
    done
    ;;
  au)
    # round 6: MobileNet 4x4 / 2x2 1x1 WGRADs -- library GEMM vs conv_wgrad_halo<1, 1> vs generic, per shape
    bash tools/gpu_steps.sh r6_au \
      lib 200 "python -u tools/probes/wgrad1x1_halo_probe.py --lib" \
      halo 200 "python -u tools/probes/wgrad1x1_halo_probe.py" \
      gen 200 "env FEDMI_WGRAD_1X1=0 python -u tools/probes/wgrad1x1_halo_probe.py"
    ;;
  av)
    # round 6: halo1-eligible 4x4 1x1 WGRADs off the library GEMM (WGRAD_GEMM_PIXELS_HALO 512) -- tests + MobileNet A/B
    bash tools/gpu_steps.sh r6_av \
      kern 300 "python -u -m pytest tests/test_cnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'wgrad_1x1'" \
      eng 400 "python -u -m pytest tests/test_kernel_list_gpu.py tests/test_cnn_native_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'launches or mobilenet or deferred'" \
      mbn1 200 "python -u bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/r6_av/mbn1.json" \
      mbn_lib 200 "python -u -c 'import sys; import fedmi.ops.conv as c; c.WGRAD_GEMM_PIXELS_HALO = 2048; sys.argv = [\"bench.py\", \"--model\", \"mobilenet\", \"--steps\", \"3\", \"--warmup\", \"1\", \"--json-out\", \"gpurun_out/r6_av/mbn_lib.json\"]; import runpy; runpy.run_path(\"bench.py\", run_name=\"__main__\")'" \
      mbn2 200 "python -u bench.py --model mobilenet --steps 3 --warmup 1 --json-out gpurun_out/r6_av/mbn2.json"
    ;;
  aw)
    # round 6: which MobileNetV2 gradients change when its 4x4 1x1 WGRADs leave the library GEMM (test failure in av)
    bash tools/gpu_steps.sh r6_aw \
      diff 200 "python -u tools/probes/halo_lib_grad_diff.py MobileNetV2"
    ;;
  ax)
    # round 6: structural-zero gradients in the MobileNetV2 tracking test (residue vs torch-bf16), then the av A/B
    bash tools/gpu_steps.sh r6_ax \
      track 300 "python -u -m pytest tests/test_cnn_native_gpu.py -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider -k 'track'"
    ;;
  ay)
    # round 6: the failover drills (GPU) with client-log tails on failure, after the suite's one 8-client drill failure
    bash tools/gpu_steps.sh r6_ay \
      drills 600 "env FEDMI_FAILOVER_REPORT=gpurun_out/r6_ay/drills.jsonl python -u -m pytest tests/test_failover_kill.py tests/test_failover_collective.py -m gpu -x -v --timeout 420 --timeout-method thread -p no:cacheprovider"
    ;;
  list) awk '/^  [a-z]+\)$/ {n=$1; getline; sub(/^ *# round 6: /, ""); print n, $0}' "$0" ;;
  *) echo "unknown run: $run (try: list)" >&2; exit 2 ;;
esac
