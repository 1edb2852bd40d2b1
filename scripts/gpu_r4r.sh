#!/bin/bash
# Round 4 (r): relaxation check interval at the 65536-bit subsequences of a
# 1000-frame call (ICX_DEC_CHECK, default 2 launches), e2e A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=2 bash scripts/ab_e2e.sh base ICX_DEC_CHECK=1 ICX_DEC_CHECK=3 ICX_DEC_WARM=6144 2>&1 | tee gpurun_out/ab_r4r_dec_check.txt
