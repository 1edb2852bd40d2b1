#!/bin/bash
# Round 5 (ah): the bit reader's window in LDS instead of registers (no
# per-step shift of the window): state-only walks (lib/libicx_ldswin.so) and
# also the write pass (lib/libicx_ldsboth.so).  Decode parity through the base
# (reader refactor, registers) and both variants, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5ah_base.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ah_base.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ah_base.log
ICX_LIB=$PWD/image-compression_amd/lib/libicx_ldsboth.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5ah_lds.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ah_lds.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ah_lds.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_ldswin.so lib/libicx_ldsboth.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_ldswin.so lib/libicx_ldsboth.so || exit 1
