#!/bin/bash
# Round 5 (af): the write step's size-0 symbols put their 0 at the end of
# their zero run (no select per put).  Decode parity, then A/B against the
# build before it (lib/libicx_prevbit.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py tests/test_cmyk_gpu.py > gpurun_out/pytest_gpu_r5af.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5af.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5af.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_prevbit.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_prevbit.so || exit 1
