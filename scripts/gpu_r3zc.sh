set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r3zc.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3zc.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r3zc.log
ROUNDS=4 timeout -k 10 600 bash scripts/ab.sh lib/libicx_prev.so base > gpurun_out/ab_r3zc_fdct_tile_row.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zc_fdct_tile_row.txt
