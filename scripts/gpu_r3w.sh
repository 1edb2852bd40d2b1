set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_pipeline_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_leanw.log 2>&1 || { tail -20 gpurun_out/pytest_leanw.log; exit 1; }
ROUNDS=3 AB_ARGS="--distinct 200" timeout -k 10 600 bash scripts/ab_decode.sh base lib/libicx_leansync.so lib/libicx_prelean.so > gpurun_out/ab_dec_leanw.txt 2>&1
