#!/bin/bash
# Round 4 (x): lean walks pick the next Huffman table from a per-block map in
# scalar registers (ICX_DEC_BSEL, lib/libicx_bs.so): decode parity with it,
# then e2e A/B against the component arithmetic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_bs.so timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_r4x.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r4x.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r4x.log
ROUNDS=2 bash scripts/ab_e2e.sh base lib/libicx_bs.so 2>&1 | tee gpurun_out/ab_r4x_dec_bsel.txt
