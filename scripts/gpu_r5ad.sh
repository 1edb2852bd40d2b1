#!/bin/bash
# Round 5 (ad): symbol-pair fields as (bits consumed, extra bits, advance)
# instead of (code length, extra bits, advance): one add and one bit-field
# extract less per state-only step.  Decode parity, then A/B against the
# previous layout (lib/libicx_prevpair.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py tests/test_cmyk_gpu.py > gpurun_out/pytest_gpu_r5ad.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ad.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ad.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_prevpair.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_prevpair.so || exit 1
