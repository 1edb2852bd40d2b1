#!/bin/bash
# Round 5 (ap): re-check the warm-up length and the subsequence length on
# today's walks (environment overrides of the defaults: 8192 warm-up bits;
# 65536 / 32768 subsequence bits at 1000 / 200 frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base ICX_DEC_WARM=4096 ICX_DEC_WARM=16384 ICX_DEC_SUB_BITS=32768 ICX_DEC_SUB_BITS=131072 || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base ICX_DEC_WARM=4096 ICX_DEC_WARM=16384 ICX_DEC_SUB_BITS=16384 ICX_DEC_SUB_BITS=65536 || exit 1
