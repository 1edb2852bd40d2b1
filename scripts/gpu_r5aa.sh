#!/bin/bash
# Round 5 (aa): two first-sync walks per lane stepped alternately
# (ICX_DEC_SYNC_ILP=1, 92 VGPRs: 5 waves x 2 chains per SIMD against 8 x 1):
# decode parity on that build, then decode A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_ilp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py tests/test_cmyk_gpu.py > gpurun_out/pytest_gpu_r5aa.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5aa.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5aa.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_ilp.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_ilp.so || exit 1
