#!/bin/bash
# Round 5 (ax): write-pass flush of two finished blocks per round (lanes
# 0..31 / 32..63, ICX_DEC_FLUSH2: lib/libicx_fl2.so) re-checked on the
# trimmed write step, against one per round (base).  Parity, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
ICX_LIB=$PWD/image-compression_amd/lib/libicx_fl2.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5ax.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ax.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ax.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_fl2.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_fl2.so || exit 1
