#!/bin/bash
# Round 5 (x): 16 checkpoint intervals for 65536-bit and longer
# subsequences (8 below) as the default build, against the previous 8
# everywhere (lib/libicx_ck8.so); GPU tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_r5x.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r5x.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5x.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_ck8.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_ck8.so || exit 1
