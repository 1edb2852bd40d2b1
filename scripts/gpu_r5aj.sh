#!/bin/bash
# Round 5 (aj): k_unstuff_count runs the byte-class masks only on the chunks
# holding a 0xFF byte, compacted into full lanes (ICX_UNSTUFF_COMPACT, base)
# against the per-lane branch (lib/libicx_nocompact.so).  Decode parity, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py tests/test_cmyk_gpu.py > gpurun_out/pytest_gpu_r5aj.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5aj.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5aj.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_nocompact.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_nocompact.so || exit 1
