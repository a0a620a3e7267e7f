#!/bin/bash
# Register/spill report of the kernels of one transform length (fast compile):
#   tools/spills.sh 13 [extra hipcc flags]
L=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -c -I"$ROOT/include" -DSW_ONLY_LOG2=$L "$@" \
  "$ROOT/juliaraytracingsw_amd/csrc/sw_kernels.hip" -o /tmp/spills.o -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c "
import re, sys
cur = None
for ln in sys.stdin:
    m = re.search(r'Function Name: (\S+)', ln)
    if m: cur = m.group(1); continue
    if cur and 'Li$L' in cur and ('VGPRs:' in ln or 'VGPRs Spill' in ln or 'Occupancy' in ln):
        print(cur[:48], ln.split('remark:')[1].strip().split(' [')[0])
"
