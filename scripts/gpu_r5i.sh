#!/bin/bash
# Round 5 (i): colour-pass occupancy (waves per SIMD 7 / 8 against the
# compiler's 6 at 74 VGPRs) and tiles per workgroup (2 / 8 against 4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_lcw7.so lib/libicx_lcw8.so lib/libicx_lct2.so lib/libicx_lct8.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh base lib/libicx_lcw7.so lib/libicx_lcw8.so lib/libicx_lct2.so lib/libicx_lct8.so || exit 1
