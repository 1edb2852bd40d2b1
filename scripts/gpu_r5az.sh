#!/bin/bash
# Round 5 (az): luma + colour tiles per workgroup 8 (loads 3 ahead,
# lib/libicx_lct8.so) and 6 (4 ahead, lct6pf4) against 4 (3 ahead, base).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
ICX_LIB=$PWD/image-compression_amd/lib/libicx_lct8.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5az.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5az.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5az.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_lct8.so lib/libicx_lct6pf4.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_lct8.so lib/libicx_lct6pf4.so || exit 1
