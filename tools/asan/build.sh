#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of the native LeNet runtime driver
# (SURVEY.md §5.2).  Only the host code is instrumented: every -fsanitize= sits behind -Xarch_host, the
# gfx950 device code is compiled normally.  Run on the GPU box with
#   ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0 ./tools/asan/bin/lenet_engine_asan
# (verify_asan_link_order=0: the box preloads a small library of its own; leaks: the HIP runtime keeps
# process-lifetime allocations).
set -eu
cd "$(dirname "$0")/../.."
out=tools/asan/bin
mkdir -p "$out"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
HIPCC=/opt/rocm/bin/hipcc
$HIPCC -O1 -g -std=c++17 --offload-arch=gfx950 $SAN -I csrc -c csrc/kernels/lenet_kernels.hip -o "$out/lenet_kernels.o"
$HIPCC -O1 -g -std=c++17 --offload-arch=gfx950 $SAN -I csrc -c csrc/runtime/lenet_engine.cpp -o "$out/lenet_engine.o"
$HIPCC -O1 -g -std=c++17 --offload-arch=gfx950 $SAN -I csrc -c tools/asan/lenet_engine_asan.cpp -o "$out/driver.o"
$HIPCC --offload-arch=gfx950 $SAN "$out/lenet_kernels.o" "$out/lenet_engine.o" "$out/driver.o" -o "$out/lenet_engine_asan"
echo "built $out/lenet_engine_asan"
