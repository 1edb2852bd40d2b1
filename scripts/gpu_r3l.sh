set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lean.log 2>&1 || { tail -20 gpurun_out/pytest_lean.log; exit 1; }
ROUNDS=3 AB_ARGS="--distinct 200" timeout -k 10 600 bash scripts/ab_decode.sh base lib/libicx_prelean.so ICX_DEC_WARM=16384 > gpurun_out/ab_dec_lean.txt 2>&1
