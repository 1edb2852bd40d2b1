#!/bin/bash
# Round 5 (an): k_dec_luma_color_420 with the tile loop unrolled, loads
# clamped instead of branched around, interior tiles on a fixed store
# sequence (ICX_DEC_LC_FULL) so the loop does not wait for its stores;
# loads 1 (base) / 2 / 3 tiles ahead (lib/libicx_f2.so, f3), and without the
# interior path (nofull).  Decode parity (base, f3), then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5an.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5an.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5an.log
ICX_LIB=$PWD/image-compression_amd/lib/libicx_f3.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5an_f3.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5an_f3.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5an_f3.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_f2.so lib/libicx_f3.so lib/libicx_nofull.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_f2.so lib/libicx_f3.so lib/libicx_nofull.so || exit 1
