#!/bin/bash
# Round 4 (h): decode parity at the new default subsequence length (32768 bits
# on large batches) with the padded luma tile; A/B of the length.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "decode or pipeline or configs" \
    > gpurun_out/pytest_gpu_r4h.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r4h.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r4h.log
ROUNDS=2 bash scripts/ab_e2e.sh base lib/libicx_ck16.so ICX_DEC_SUB_BITS=16384 ICX_DEC_SUB_BITS=65536 2>&1 | tee gpurun_out/ab_r4h_dec_sub.txt
