#!/bin/bash
# Round 5 (av): 16 checkpoint intervals (2048 bits) for 32768-bit
# subsequences too (lib/libicx_cks16.so) against 8 (base): the 200- and
# 64-frame calls.  Decode parity on the variant, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
ICX_LIB=$PWD/image-compression_amd/lib/libicx_cks16.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5av.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5av.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5av.log
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_cks16.so || exit 1
echo "== 64 frames"
FRAMES=64 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_cks16.so || exit 1
