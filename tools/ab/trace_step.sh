export TMPDIR=/tmp
mkdir -p gpurun_out/tr
SW_PRE_PER_CU=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr/t1 -o run -- python tools/prof_step.py --steps 10 --warmup 3 > gpurun_out/tr/t1.log 2>&1 || exit 1
cp $(find gpurun_out/tr/t1 -name '*kernel_trace.csv') gpurun_out/tr/kt1.csv
