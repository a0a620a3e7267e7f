#!/bin/bash
# On the GPU box (round 4): half-length rows — rows per block (SW_ROWH_NB,
# SW_RSW_ROWH_NB) and the RSW half row's single read of V (SW_RSW_ROWH_ZPARK):
# interleaved benches of sweep_var/q13*.so (config 5) and r12*.so (config 4),
# then PMC traffic per variant (tools/traffic_at.sh).
# usage: bash tools/ab/ab_r4_rowh.sh [R]
mkdir -p gpurun_out/ab
R=${1:-2}
run() {  # name model grid stepper steps warmup
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 \
    --model $2 --grid $3 --stepper $4 --steps $5 --warmup $6 > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err \
    || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in $(seq $R); do
  for v in $(ls sweep_var | grep '^q13' | sed 's/.so$//'); do run $v qg2 8192 IFMRK4 12 3 || exit 1; done
  for v in $(ls sweep_var | grep '^r12' | sed 's/.so$//'); do run $v rsw 4096 FilteredAB3 100 20 || exit 1; done
done
for v in $(ls sweep_var | grep "^q13" | sed "s/.so$//"); do bash tools/traffic_at.sh $PWD/sweep_var/$v.so $v qg2 IFMRK4 8192 4 || exit 2; done
for v in $(ls sweep_var | grep '^r12' | sed 's/.so$//'); do bash tools/traffic_at.sh $PWD/sweep_var/$v.so $v rsw FilteredAB3 4096 10 || exit 3; done
for f in gpurun_out/tr/*/t.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', {k: (round(d['fetch_bytes'].get(k,0)/1e6,1), round(d['write_bytes'].get(k,0)/1e6,1)) for k in d['kernels']})"; done
