set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ev; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bench -o run -- \
  python bench.py --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || exit 2
cp $(find $O/trace_bench -name '*kernel_stats.csv') $O/kernel_stats_bench.csv || exit 3
rm -rf $O/trace_bench
SW_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --steps 10 --warmup 2 --no-config5 \
  --config4-steps 3 --no-cpu-baseline --no-cold-profile > $O/bench_gloo8_rehearsal.json 2> $O/bench_gloo8.err \
  || { tail -20 $O/bench_gloo8.err; exit 4; }
python -c "import json; b=json.load(open('$O/bench_gloo8_rehearsal.json')); print(b['n_gpus'], b['config']['parallelism'], b['slab_error'], b['config4']['n_gpus'], b['config4']['ranks_idle'], b['config4']['value'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driverlike.json 2> $O/bench_driverlike.err || exit 5
python -c "import json; b=json.load(open('$O/bench_driverlike.json')); print('driverlike', round(b['value'],1), round(b['ms_per_step']*1e3,2), [(k['name'], round(k['avg_us'],1)) for k in b['kernels']])"
