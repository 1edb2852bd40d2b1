#!/bin/bash
# Round 5 (ae): the long-code test of every walk step as one bit test
# (DEC_LEAN_LONG, a zig-zag advance no symbol has) instead of "no bits
# consumed and not invalid".  Decode parity, then A/B against the build
# before it (lib/libicx_paironly.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py tests/test_cmyk_gpu.py > gpurun_out/pytest_gpu_r5ae.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ae.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ae.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_paironly.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_paironly.so || exit 1
