#!/bin/bash
# Round 5 (aw): FDCT tiles per workgroup 2 (lib/libicx_ft2.so; 4 does not build: the writelane asm runs out of SGPR operands)
# against 3 (base) now that a tile's stores no longer hold up the next
# tile's pixels.  Encode parity (ft2), then the headline A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ICX_LIB=$PWD/image-compression_amd/lib/libicx_ft2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_gpu_r5aw.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5aw.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5aw.log
ROUNDS=4 bash scripts/ab.sh base lib/libicx_ft2.so || exit 1
