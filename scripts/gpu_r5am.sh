#!/bin/bash
# Round 5 (am): k_dec_luma_color_420 with its tile loop unrolled and the loads
# of 2 / 3 tiles ahead in flight (lib/libicx_pf2.so, pf3; pf2t8: 8 tiles per
# workgroup) against one tile ahead (base).  Decode parity (pf2), then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
ICX_LIB=$PWD/image-compression_amd/lib/libicx_pf2.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5am_pf2.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5am_pf2.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5am_pf2.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_pf2.so lib/libicx_pf3.so lib/libicx_pf2t8.so || exit 1
