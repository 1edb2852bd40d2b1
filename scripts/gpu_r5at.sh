#!/bin/bash
# Round 5 (at): k_dec_idct (chroma IDCT) with several tiles per workgroup,
# loads 1-3 tiles ahead and one store per lane on every path (dummy blocks to
# the planes' spare bytes): lib/libicx_i2p1.so (2 tiles, 1 ahead), i4p2, i4p3,
# against one tile per workgroup (base).  Decode parity on each variant, A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_decode_gpu.py tests/test_cmyk_gpu.py"
timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5at.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5at.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5at.log
for v in i2p1 i4p3; do
  ICX_LIB=$PWD/image-compression_amd/lib/libicx_$v.so timeout -k 10 300 $T > gpurun_out/pytest_gpu_r5at_$v.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5at_$v.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu_r5at_$v.log
done
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=3 bash scripts/ab_decode.sh base lib/libicx_i2p1.so lib/libicx_i4p2.so lib/libicx_i4p3.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_i2p1.so lib/libicx_i4p2.so lib/libicx_i4p3.so || exit 1
