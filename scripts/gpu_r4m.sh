#!/bin/bash
# Round 4 (m): k_huff with the chunk's blocks dealt by descending list length
# (ICX_HUFF_SORT): encode parity with that build, then the headline A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_hs.so timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py \
    tests/test_configs_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4m.log 2>&1 \
    || { tail -30 gpurun_out/pytest_gpu_r4m.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r4m.log
IMAGES=1000 STEPS=6 ROUNDS=3 bash scripts/ab.sh base lib/libicx_hs.so 2>&1 | tee gpurun_out/ab_r4m_huff_sort.txt
