set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r3zk.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3zk.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r3zk.log
ROUNDS=4 AB_ARGS="--distinct 200" timeout -k 10 900 bash scripts/ab_decode.sh lib/libicx_agg0.so base > gpurun_out/ab_r3zk_dec_agg.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zk_dec_agg.txt
ROUNDS=4 timeout -k 10 900 bash scripts/ab.sh base lib/libicx_h7p32.so lib/libicx_h6p40.so > gpurun_out/ab_r3zk_huff_pre.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zk_huff_pre.txt
