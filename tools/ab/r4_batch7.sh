#!/bin/bash
# Round 4 GPU batch 7: mixed-field tile shapes at 2048 (RSW metric, 2LQG
# config 3): m11base (2x4 tiles both ways), m11ti4 (inverse tiles 4x2,
# -DSW_TILE_I=4), and m11base with SW_TILE_FA=2 (forward tiles 4x2).
mkdir -p gpurun_out/ab
for cfg in "m11ti4 SW_TILE_FA=1" "m11base SW_TILE_FA=2"; do
  set -- $cfg
  env $2 LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "2048" \
    --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$1_$2.txt 2>&1; rc=$?
  echo "$1 $2 parity rc=$rc: $(tail -1 gpurun_out/gpu_tests_$1_$2.txt)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
run() {  # tag so env model grid stepper steps warmup
  env $3 SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $4 --grid $5 --stepper $6 --steps $7 --warmup $8 \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err \
    || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2; do
  run t_base_m m11base SW_TILE_FA=1 rsw 2048 FilteredAB3 2000 200 || exit 1
  run t_ti4_m m11ti4 SW_TILE_FA=1 rsw 2048 FilteredAB3 2000 200 || exit 1
  run t_fa2_m m11base SW_TILE_FA=2 rsw 2048 FilteredAB3 2000 200 || exit 1
  run t_base_q m11base SW_TILE_FA=1 qg2 2048 IFMAB3 2000 200 || exit 1
  run t_ti4_q m11ti4 SW_TILE_FA=1 qg2 2048 IFMAB3 2000 200 || exit 1
  run t_fa2_q m11base SW_TILE_FA=2 qg2 2048 IFMAB3 2000 200 || exit 1
done
