#!/bin/bash
# Round 4 (u): one-pass unstuffing with a decoupled look-back (ICX_DEC_ONEPASS):
# the stream check on three golden files, decode and pipeline parity with that
# build, then the e2e A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ICX_DEC_DEBUG_UNSTUFF=1 ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_op.so timeout -k 10 120 python scripts/dbg_unstuff.py \
    > gpurun_out/dbg_r4u.txt 2>&1 || { tail -20 gpurun_out/dbg_r4u.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/dbg_r4u.txt | grep -v "   tile" | tail -4
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_op.so timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py \
    tests/test_pipeline_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_r4u.log 2>&1 \
    || { tail -40 gpurun_out/pytest_gpu_r4u.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r4u.log
ROUNDS=2 bash scripts/ab_e2e.sh base lib/libicx_op.so 2>&1 | tee gpurun_out/ab_r4u_dec_onepass.txt
