set -o pipefail
mkdir -p gpurun_out/r05
(timeout 60 amd-smi static -g 0 --json > gpurun_out/r05/amdsmi_static.json 2>&1; echo rc=$?) 
(timeout 60 amd-smi metric -g 0 --json > gpurun_out/r05/amdsmi_metric.json 2>&1; echo rc=$?)
(timeout 30 amd-smi partition --json > gpurun_out/r05/amdsmi_partition.json 2>&1; echo rc=$?)
(timeout 30 rocm-smi --showclocks --showpower --showmaxpower --json > gpurun_out/r05/rocmsmi.json 2>&1; echo rc=$?)
python -c "import amdsmi; print('amdsmi py ok')" 2>&1 | tail -1
timeout -k 10 300 python bench.py > gpurun_out/r05/bench_start.json 2> gpurun_out/r05/bench_start.err
echo bench rc=$?
tail -c 600 gpurun_out/r05/bench_start.json
