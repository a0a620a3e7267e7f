set -o pipefail
mkdir -p gpurun_out/ab
bash tools/ab/ab.sh 2 --grid 1024 --steps 8000 --warmup 400 --nutune 2.5 --cfltune 0.005 > gpurun_out/ab/ab1024.log 2>&1 || exit 1
export TMPDIR=/tmp
for v in noxcd xcd; do
  LIBSW_PATH=$PWD/sweep_var/$v.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ab/pf_$v -o run -- python tools/prof_step.py --grid 1024 --steps 200 --nutune 2.5 --cfltune 0.005 > gpurun_out/ab/pf_$v.log 2>&1 || exit 2
  LIBSW_PATH=$PWD/sweep_var/$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ab/pw_$v -o run -- python tools/prof_step.py --grid 1024 --steps 200 --nutune 2.5 --cfltune 0.005 > gpurun_out/ab/pw_$v.log 2>&1 || exit 3
  python tools/traffic_from_pmc.py $(find gpurun_out/ab/pf_$v -name '*counter_collection.csv') $(find gpurun_out/ab/pw_$v -name '*counter_collection.csv') rsw1024_FilteredAB3 gpurun_out/ab/traffic_$v.json > /dev/null || exit 4
  rm -rf gpurun_out/ab/pf_$v gpurun_out/ab/pw_$v
done
