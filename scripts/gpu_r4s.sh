#!/bin/bash
# Round 4 (s): k_huff without exec-mask branches on the common coded-entry
# path (branch-free slot writes ICX_HUFF_PUT_NB, wave-uniform zero-run test
# ICX_HUFF_ZRL_ANY): encode parity with both, headline A/B; then the decode
# relaxation check interval (ICX_DEC_CHECK) on the e2e leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_nbza.so timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py \
    tests/test_configs_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4s.log 2>&1 \
    || { tail -30 gpurun_out/pytest_gpu_r4s.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r4s.log
IMAGES=1000 STEPS=6 ROUNDS=2 bash scripts/ab.sh base lib/libicx_nb.so lib/libicx_za.so lib/libicx_nbza.so 2>&1 \
    | tee gpurun_out/ab_r4s_huff_branch.txt || exit 1
ROUNDS=2 bash scripts/ab_e2e.sh base ICX_DEC_CHECK=1 ICX_DEC_CHECK=3 2>&1 | tee gpurun_out/ab_r4s_dec_check.txt
