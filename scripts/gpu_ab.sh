#!/bin/bash
# GPU-box helper for a decoder A/B: the GPU tests on the default build, then
# scripts/ab_decode.sh over 1000 frames (16 distinct sources) for the default
# library and VARIANTS (ab_decode.sh's forms), and with E2E=1 the e2e leg
# (scripts/ab_e2e.sh, 1000 distinct sources).  Each step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
  tail -1 gpurun_out/pytest_ab.log
fi
FRAMES=${FRAMES:-1000} STEPS=3 AB_ARGS="--distinct 16" ROUNDS=${ROUNDS:-2} timeout -k 10 600 bash scripts/ab_decode.sh base ${VARIANTS} > gpurun_out/ab_dec.txt 2>&1 || { tail -5 gpurun_out/ab_dec.txt; exit 1; }
cat gpurun_out/ab_dec.txt
if [ -n "$E2E" ]; then
  ROUNDS=${ROUNDS:-2} timeout -k 10 700 bash scripts/ab_e2e.sh base ${VARIANTS} > gpurun_out/ab_e2e.txt 2>&1 || { tail -5 gpurun_out/ab_e2e.txt; exit 1; }
  cat gpurun_out/ab_e2e.txt
fi
