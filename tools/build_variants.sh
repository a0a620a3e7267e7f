#!/bin/bash
# Build libsw variants with extra -D flags into sweep_var/<name>.so (perf sweeps).
# usage: tools/build_variants.sh name1:"-DFOO=1" name2:"-DBAR=2" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/sweep_var"
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -Wno-unused-result \
    -I"$ROOT/include" $flags -o "$ROOT/sweep_var/$name.so" \
    "$ROOT/juliaraytracingsw_amd/csrc/sw_kernels.hip" "$ROOT/juliaraytracingsw_amd/csrc/sw_api.cpp" \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la "$ROOT/sweep_var"
