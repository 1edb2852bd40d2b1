#!/bin/bash
# Round 5 (w): checkpoint intervals per subsequence (ICX_DEC_CK_DIV 16 / 4
# against 8): a relaunch re-walk stops at the first checkpoint its previous
# walk had already synchronised by, and the write pass splits subsequences at
# the checkpoints (twice / half the pieces).  r1 at 1000 frames re-walks 22 %
# of the subsequences (206k of 953k, bench_decode sync_walks_per_step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_ck16.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py > gpurun_out/pytest_gpu_r5w.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5w.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5w.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_ck16.so lib/libicx_ck4.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_ck16.so lib/libicx_ck4.so || exit 1
