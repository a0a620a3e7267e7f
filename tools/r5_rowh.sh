# round 5: the paired half rows — 4096/8192 tests on the default build, then
# config 4 (h0/h1, --len 12) and config 5 (q0/q1, --len 13) interleaved
set -o pipefail
TESTS="4096 or 8192 or large or rectangular or invariants" AB="h0 h1" BARGS="--grid 4096 --steps 400 --warmup 50" \
  R=3 bash tools/r5_ab.sh || exit 1
TESTS="" AB="q0 q1" BARGS="--model qg2 --stepper IFMRK4 --grid 8192 --steps 20 --warmup 3" R=3 bash tools/r5_ab.sh || exit 2
