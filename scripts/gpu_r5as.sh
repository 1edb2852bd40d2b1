#!/bin/bash
# Round 5 (as): FDCT list stores two per lane and group on every path (no
# rare-path branch: lib/libicx_static2.so) against one plus a rare branch
# (base).  Encode parity tests, then the headline A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ICX_LIB=$PWD/image-compression_amd/lib/libicx_static2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_gpu_r5as.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5as.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5as.log
ROUNDS=4 bash scripts/ab.sh base lib/libicx_static2.so || exit 1
