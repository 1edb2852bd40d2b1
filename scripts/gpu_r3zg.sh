set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r3zg.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3zg.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r3zg.log
ROUNDS=5 timeout -k 10 900 bash scripts/ab.sh lib/libicx_prev.so base lib/libicx_st0.so lib/libicx_noat.so > gpurun_out/ab_r3zg_fdct_lds.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zg_fdct_lds.txt
