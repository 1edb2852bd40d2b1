set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r3z.log 2>&1 || exit 1
ROUNDS=2 AB_ARGS="--distinct 200" timeout -k 10 500 bash scripts/ab_decode.sh base ICX_DEC_CHECK=1 ICX_DEC_CHECK=3 > gpurun_out/ab_dec_check.txt 2>&1
