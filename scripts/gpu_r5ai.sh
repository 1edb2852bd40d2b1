#!/bin/bash
# Round 5 (ai): LDS window of the state-only walks on by default (base);
# window of 6 / 12 words against 8 (lib/libicx_win6.so, lib/libicx_win12.so:
# LDS per workgroup 23 / 29 KiB against 25).  Decode + full GPU parity on the
# base, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_gpu_r5ai.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ai.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ai.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_win6.so lib/libicx_win12.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_win6.so lib/libicx_win12.so || exit 1
