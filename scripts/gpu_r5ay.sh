#!/bin/bash
# Round 5 (ay): 32 checkpoint intervals per 65536-bit subsequence (write-pass
# pieces of 2048 bits; lib/libicx_ck32.so) against 16 (base).  Parity, A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
ICX_LIB=$PWD/image-compression_amd/lib/libicx_ck32.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5ay.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ay.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ay.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_ck32.so || exit 1
