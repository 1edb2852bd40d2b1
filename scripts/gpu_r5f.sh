#!/bin/bash
# Round 5 (f): decoder parameter re-tune after the symbol pairs (env-only
# A/B: subsequence length, warm-up length, sync launches per check).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base ICX_DEC_SUB_BITS=32768 ICX_DEC_SUB_BITS=131072 ICX_DEC_WARM=4096 ICX_DEC_WARM=12288 ICX_DEC_CHECK=3 lib/libicx_lcdw.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base ICX_DEC_SUB_BITS=16384 ICX_DEC_SUB_BITS=65536 ICX_DEC_WARM=4096 ICX_DEC_WARM=12288 ICX_DEC_CHECK=1 lib/libicx_lcdw.so || exit 1
