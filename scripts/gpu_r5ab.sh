#!/bin/bash
# Round 5 (ab): window words of the state-only walks (ICX_DEC_WIN 4 / 6 / 12
# against 8): each step's refill shifts the window with WIN-1 selects, a
# shorter window refills from HBM more often.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_win4.so lib/libicx_win6.so lib/libicx_win12.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh base lib/libicx_win4.so lib/libicx_win6.so lib/libicx_win12.so || exit 1
