#!/bin/bash
# Round 5 (v): write-pass A/B after the symbol pairs and the 9-bit look-ups:
# two finished blocks per flush round (ICX_DEC_FLUSH2), write window 7 / 12
# words against 9, one step per top-up check (ICX_DEC_WRITE_UNROLL2=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_flush2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py > gpurun_out/pytest_gpu_r5v.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5v.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5v.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_flush2.so lib/libicx_ww7.so lib/libicx_ww12.so lib/libicx_wu1.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh base lib/libicx_flush2.so lib/libicx_ww7.so lib/libicx_ww12.so lib/libicx_wu1.so || exit 1
