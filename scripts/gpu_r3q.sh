set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_predw.log 2>&1 || { tail -20 gpurun_out/pytest_predw.log; exit 1; }
ROUNDS=3 AB_ARGS="--distinct 200" timeout -k 10 900 bash scripts/ab_decode.sh base lib/libicx_pred.so lib/libicx_win4.so lib/libicx_win6.so > gpurun_out/ab_dec_predw.txt 2>&1
