#!/bin/bash
# Round 5 (ba): state-only walks in 512-thread workgroups (the 16 KiB of
# tables shared by 8 waves: 34 KiB per workgroup, 8 waves per SIMD instead
# of 6; lib/libicx_nt512.so) against 256 (base).  Parity, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
ICX_LIB=$PWD/image-compression_amd/lib/libicx_nt512.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5ba.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ba.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ba.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_nt512.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_nt512.so || exit 1
echo "== 64 frames"
FRAMES=64 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_nt512.so || exit 1
