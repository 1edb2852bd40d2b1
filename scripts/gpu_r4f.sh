#!/bin/bash
# Round 4 (f): decode parity with the reverted IDCT / scatter tiling, then an
# A/B of the decoder's tile-per-workgroup counts on the e2e leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "decode or pipeline" \
    > gpurun_out/pytest_gpu_r4f.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r4f.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r4f.log
ROUNDS=2 bash scripts/ab_e2e.sh lib/libicx_b.so lib/libicx_c1.so lib/libicx_lc1.so lib/libicx_lc2.so lib/libicx_lc8.so \
    lib/libicx_i2.so 2>&1 | tee gpurun_out/ab_r4f_dec_tiles.txt
