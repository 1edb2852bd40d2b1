#!/bin/bash
# Round 5 (k): unstuffing tiling A/B - k_unstuff_count 2.80 ms (2.8 TB/s on
# 7.81 GB) and k_unstuff_scatter 5.16 ms (3.0 TB/s on 15.6 GB) per 1000
# frames (rocprof_r5j_dec1000): tiles per count workgroup 2 / 8 against 4,
# tiles per scatter workgroup 2 against 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_ut2.so lib/libicx_ut8.so lib/libicx_st2.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh base lib/libicx_ut2.so lib/libicx_ut8.so lib/libicx_st2.so || exit 1
