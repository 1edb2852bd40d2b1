#!/bin/bash
# Round 4 (g): A/B of the write pass (two-block flush, scalar-cache second
# levels) and of the subsequence / warm-up lengths on the e2e leg; then SQ
# counters of the decoder (200 4K q95 frames, 8 distinct).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=2 bash scripts/ab_e2e.sh base lib/libicx_s2.so lib/libicx_f2.so ICX_DEC_WARM=4096 ICX_DEC_SUB_BITS=32768 \
    2>&1 | tee gpurun_out/ab_r4g_dec.txt || exit 1
TAG=sq_r4g SQ_PROG=scripts/bench_decode.py SQ_ARGS="--frames 200 --distinct 8 --steps 1 --warmup 0" T_SQ=240 \
    ICX_LIBS="image-compression_amd/lib/libicx.so image-compression_amd/lib/libicx_s2.so" \
    bash scripts/gpu_sq.sh > gpurun_out/sq_r4g_decode.txt 2>&1 || { tail -20 gpurun_out/sq_r4g_decode.txt; exit 1; }
grep -A16 "k_dec_write" gpurun_out/sq_r4g_decode.txt | head -40
