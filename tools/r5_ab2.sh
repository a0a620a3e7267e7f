# round 5: bitwise state hash of each sweep_var/<name>.so in $AB, then the
# interleaved benches (tools/r5_ab.sh)
set -o pipefail
for so in $AB; do LIBSW_PATH=$PWD/sweep_var/$so.so timeout -k 10 120 python tools/state_hash.py 10 || exit 5; done
bash tools/r5_ab.sh
