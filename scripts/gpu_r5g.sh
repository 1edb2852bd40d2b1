#!/bin/bash
# Round 5 (g): colour pass and IDCT on full-rate 24-bit products (v_mad_i32_i24
# instead of the quarter-rate v_mul_lo_u32 / v_mad_u64_u32 the compiler chose),
# edge chroma columns replicated at staging (no edge cases in the colour
# pass), 8 second-level Huffman tables.  Decode parity first, then A/B against
# the previous colour pass (lib/libicx_nsub8.so: same tree before the change).
# (r5g: the first build failed parity - the compiler had packed clamped bytes
# with its own v_ashr_pk_u8_i32 and ORed the result as if its high half were
# zero; the packing is now explicit.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py tests/test_cmyk_gpu.py > gpurun_out/pytest_gpu_${TAG:-r5g}.log 2>&1 \
    || { tail -30 gpurun_out/pytest_gpu_${TAG:-r5g}.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_${TAG:-r5g}.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_nsub8.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_nsub8.so || exit 1
