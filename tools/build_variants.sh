#!/bin/bash
# Build libsw variants with extra -D flags into sweep_var/<name>.so (perf sweeps).
# usage: tools/build_variants.sh [--len L] name1:"-DFOO=1" name2:"-DBAR=2" ...
#   --len L: build transform length 2^L only (fast; benches at that grid only)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/sweep_var"
LEN=None
if [ "$1" = "--len" ]; then LEN="[$2]"; shift 2; fi
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  python3 -c "
import sys; sys.path.insert(0, '$ROOT')
from juliaraytracingsw_amd import build
print(build.build_lib(force=True, out='$ROOT/sweep_var/$name.so', extra_flags=['-DSW_EXPERIMENTS'] + '$flags'.split(), parts=$LEN))"
done
ls -la "$ROOT/sweep_var"
