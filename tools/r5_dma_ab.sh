# round 5: the LDS-DMA RSW row — bitwise/parity tests, the checkpoint and
# scipy-expm parity changes, then an interleaved A/B of SW_ROW_DMA=1
# (k_row_rsw_dma) against SW_ROW_DMA=0 (k_row)
set -o pipefail
O=gpurun_out/r05/dma; mkdir -p $O
python -c "import sys; sys.exit(0 if b'k_row_rsw_dma' in open('juliaraytracingsw_amd/libsw.so','rb').read() else 1)" || { echo "stale libsw.so"; exit 3; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_aliased.py tests/test_gpu_large.py \
  -k "row_dma or large or determinism or checkpoint or config5" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2 3; do for d in 1 0; do
  SW_ROW_DMA=$d timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-box-state \
    --steps 2000 --warmup 200 > $O/b$d.$r.json 2> $O/b$d.$r.err || { echo "bench $d failed"; tail $O/b$d.$r.err; exit 2; }
  echo "r$r dma=$d $(python -c "import json; d=json.load(open('$O/b$d.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
