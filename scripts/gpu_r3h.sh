set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_huffasm.log 2>&1 || { tail -20 gpurun_out/pytest_huffasm.log; exit 1; }
ROUNDS=3 timeout -k 10 600 bash scripts/ab.sh base lib/libicx_orall.so > gpurun_out/ab_huff_asm.txt 2>&1
