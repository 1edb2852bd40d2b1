#!/bin/bash
# Round 5 (ao): k_fdct_color with loads and stores the compiler counts on
# every path (ICX_FDCT_STATIC: pixel loads unconditional, thresholds loaded
# with the tile's pixels, zig-zag index once per workgroup, one list store
# per group and lane, meta stores global not flat, no register copies between
# tiles) against the round's previous FDCT (lib/libicx_static0.so).  All GPU
# tests on the base, then the headline A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_gpu_r5ao.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5ao.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5ao.log
ROUNDS=4 bash scripts/ab.sh base lib/libicx_static0.so || exit 1
