#!/bin/bash
# Round 4 (t): k_unstuff_count with 8 / 16 tiles per workgroup, e2e A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_c16.so timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -x -q \
    -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4t.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r4t.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r4t.log
ROUNDS=2 bash scripts/ab_e2e.sh base lib/libicx_c8.so lib/libicx_c16.so 2>&1 | tee gpurun_out/ab_r4t_dec_count.txt
