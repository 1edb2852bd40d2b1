#!/bin/bash
# Round 5 (ak): k_unstuff_scatter computes the byte-class masks on compacted
# special chunks (ICX_SCATTER_COMPACT, base: 1 tile per workgroup;
# lib/libicx_sc2.so / sc4.so: 2 / 4 tiles per workgroup, where the compaction
# runs the masks once for all of them) against the per-lane masks
# (lib/libicx_scold.so).  Decode parity (base, sc4), then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5ak.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ak.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ak.log
ICX_LIB=$PWD/image-compression_amd/lib/libicx_sc4.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5ak_sc4.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ak_sc4.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ak_sc4.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_sc2.so lib/libicx_sc4.so lib/libicx_scold.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_sc2.so lib/libicx_sc4.so lib/libicx_scold.so || exit 1
