#!/bin/bash
# Round 5 (ag): state-only walks run an unpredicated loop while every lane
# of the wave walks (ICX_DEC_WALK_ALL, lib/libicx_walkall.so).  Decode
# parity through the variant, then A/B against the base build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ICX_LIB=$PWD/image-compression_amd/lib/libicx_walkall.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py tests/test_cmyk_gpu.py > gpurun_out/pytest_gpu_r5ag.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ag.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ag.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_walkall.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_walkall.so || exit 1
