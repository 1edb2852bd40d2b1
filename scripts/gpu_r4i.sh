#!/bin/bash
# Round 4 (i): subsequence length, warm-up and checkpoint count on the e2e leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=2 bash scripts/ab_e2e.sh ICX_DEC_SUB_BITS=65536 ICX_DEC_SUB_BITS=131072 ICX_DEC_SUB_BITS=65536,ICX_DEC_WARM=16384 \
    lib/libicx_ck4.so:ICX_DEC_SUB_BITS=65536 lib/libicx_ck4.so:ICX_DEC_SUB_BITS=16384 2>&1 | tee gpurun_out/ab_r4i_dec_sub.txt
