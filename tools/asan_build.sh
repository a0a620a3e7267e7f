#!/bin/bash
# Host-only AddressSanitizer build of the C-ABI runtime plus its driver
# (tests/abi_asan.cpp): sw_api.cpp and the driver instrumented, the device
# kernels (64-point length only) built normally.  Output: tests/asan_bin/abi_asan
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O=$ROOT/tests/asan_bin
mkdir -p $O
rm -f $O/*.o $O/abi_asan  # never link objects left by an earlier build
H=/opt/rocm/bin/hipcc
C="-O1 -g -std=c++17 --offload-arch=gfx950 -I$ROOT/include -I$ROOT/juliaraytracingsw_amd/csrc"
pids=()
$H $C -DSW_ONLY_LOG2=6 -DSW_PART=0 -c $ROOT/juliaraytracingsw_amd/csrc/sw_kernels.hip -o $O/k0.o & pids+=($!)
$H $C -DSW_ONLY_LOG2=6 -DSW_PART=6 -c $ROOT/juliaraytracingsw_amd/csrc/sw_kernels.hip -o $O/k6.o & pids+=($!)
$H $C -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -c $ROOT/juliaraytracingsw_amd/csrc/sw_api.cpp -o $O/api.o & pids+=($!)
$H $C -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -c $ROOT/tests/abi_asan.cpp -o $O/drv.o & pids+=($!)
$H $C -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -c $ROOT/juliaraytracingsw_amd/csrc/sw_generic.hip -o $O/gen.o & pids+=($!)
# a bare `wait` returns 0 even when a compile failed: wait for each one
for pid in "${pids[@]}"; do wait "$pid" || { echo "asan_build: a compile failed" >&2; exit 1; }; done
$H --offload-arch=gfx950 -fsanitize=address -fno-gpu-sanitize -o $O/abi_asan $O/drv.o $O/api.o $O/gen.o $O/k0.o $O/k6.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo $O/abi_asan
