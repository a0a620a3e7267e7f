#!/bin/bash
# Round 4 GPU batch 12: pruned decimated row transforms on/off at 2048
# (m11base / m11np, -DSW_ROW_PRUNE=0), the paired 2LQG col_inv at 2048
# (m11pair, -DSW_QG_INV_PAIR=2), then the N=2 bench line rehearsed on
# one GPU over gloo (host-staged slab transport).
mkdir -p gpurun_out/ab
run() {  # tag so model grid stepper steps warmup
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2 3; do
  run p_base_m m11base rsw 2048 FilteredAB3 2000 200 || exit 1
  run p_np_m m11np rsw 2048 FilteredAB3 2000 200 || exit 1
  run p_base_q m11base qg2 2048 IFMAB3 2000 200 || exit 1
  run p_np_q m11np qg2 2048 IFMAB3 2000 200 || exit 1
  run p_pair_q m11pair qg2 2048 IFMAB3 2000 200 || exit 1
done
SW_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo "gloo2 failed"; tail -20 gpurun_out/bench_gloo2.err; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/bench_gloo2.json')); print({k: d[k] for k in ('value','n_gpus','scaling','config')}); print(json.dumps(d.get('comm'))[:600])"
