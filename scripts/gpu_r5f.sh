#!/bin/bash
# Round 5 (f): decoder A/B after the symbol pairs: 8 second-level tables per
# Huffman table (sync / init LDS 24 -> 16 KiB), dword chroma reads in the
# colour pass, and env-only parameters (subsequence length, warm-up, checks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== builds, 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_nsub8.so lib/libicx_lcdw.so lib/libicx_nsub8lc.so || exit 1
echo "== write-pass workgroup size with split tails, 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh base ICX_DEC_TAIL_SPLIT=2 lib/libicx_nt320.so lib/libicx_nt320.so:ICX_DEC_TAIL_SPLIT=2 lib/libicx_nt448.so:ICX_DEC_TAIL_SPLIT=2 || exit 1
echo "== builds, 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_nsub8.so lib/libicx_lcdw.so lib/libicx_nsub8lc.so || exit 1
echo "== parameters, 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh base ICX_DEC_SUB_BITS=32768 ICX_DEC_SUB_BITS=131072 ICX_DEC_WARM=4096 ICX_DEC_WARM=12288 ICX_DEC_CHECK=1 ICX_DEC_CHECK=3 || exit 1
echo "== parameters, 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh base ICX_DEC_SUB_BITS=16384 ICX_DEC_SUB_BITS=65536 ICX_DEC_WARM=4096 ICX_DEC_WARM=12288 ICX_DEC_CHECK=1 || exit 1
