#!/bin/bash
# Round 5 close (2): GPU tests and smoke() on the tree as committed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r5final2.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5final2.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5final2.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' || exit 1
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh base || exit 1
