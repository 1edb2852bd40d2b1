set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r3zb.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3zb.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r3zb.log
ROUNDS=4 timeout -k 10 600 bash scripts/ab.sh lib/libicx_la0.so base > gpurun_out/ab_r3zb_fdct_emit_la.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zb_fdct_emit_la.txt
