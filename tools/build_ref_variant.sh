#!/bin/bash
# Build libsw from a git revision (default HEAD) into sweep_var/<name>.so, for
# same-box A/B sweeps against the working tree.  usage: tools/build_ref_variant.sh name [rev]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=${2:-HEAD}
wt=$(mktemp -d /tmp/swref.XXXX)
git -C "$ROOT" worktree add -q --detach "$wt" "$rev"
mkdir -p "$ROOT/sweep_var"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -Wno-unused-result \
  -I"$wt/include" -o "$ROOT/sweep_var/$name.so" \
  "$wt/juliaraytracingsw_amd/csrc/sw_kernels.hip" "$wt/juliaraytracingsw_amd/csrc/sw_api.cpp" \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
git -C "$ROOT" worktree remove --force "$wt"
