#!/bin/bash
# On the GPU box: per-kernel times of every sweep_var/*.so at the large
# configurations.  usage: bash tools/ab/sweep_sizes.sh "model stepper n steps" ...
mkdir -p gpurun_out/sizes
CFGS=("$@")
for so in sweep_var/*.so; do
  v=$(basename $so .so)
  for cfg in "${CFGS[@]}"; do
    read -r m st n k <<< "$cfg"
    f=gpurun_out/sizes/${v}_${m}_${st}_$n
    LIBSW_PATH=$PWD/$so timeout -k 10 200 python bench.py --no-cpu-baseline --model $m --stepper $st --grid $n \
      --steps $k --warmup 2 --profile-steps 3 > $f.json 2> $f.err || { echo "$v $cfg failed"; tail -3 $f.err; exit 1; }
    echo "$v $cfg $(python -c "import json; d=json.load(open('$f.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done
