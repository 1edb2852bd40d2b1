set -o pipefail
# parity of the packed FDCT phases, then an A/B against the previous kernels
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r3za.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3za.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r3za.log
ROUNDS=3 timeout -k 10 600 bash scripts/ab.sh lib/libicx_pk0.so lib/libicx_pkcol.so base > gpurun_out/ab_r3za_fdct_packed.txt 2>&1 || exit 1
cat gpurun_out/ab_r3za_fdct_packed.txt
