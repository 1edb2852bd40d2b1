#!/bin/bash
# Round 4 (g): SQ counters of the device decoder (200 4K q95 frames, 8 distinct).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=sq_r4g SQ_PROG=scripts/bench_decode.py SQ_ARGS="--frames 200 --distinct 8 --steps 1 --warmup 0" T_SQ=240 \
    bash scripts/gpu_sq.sh > gpurun_out/sq_r4g_decode.txt 2>&1 || { tail -20 gpurun_out/sq_r4g_decode.txt; exit 1; }
grep -A16 "k_dec_write\|k_dec_sync\|k_dec_init" gpurun_out/sq_r4g_decode.txt | head -80
ROUNDS=2 bash scripts/ab_e2e.sh base lib/libicx_f2.so ICX_DEC_WARM=4096 ICX_DEC_WARM=12288 ICX_DEC_SUB_BITS=32768 ICX_DEC_SUB_BITS=8192 \
    2>&1 | tee gpurun_out/ab_r4g_dec_sub.txt
