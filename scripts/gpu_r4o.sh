#!/bin/bash
# Round 4 (o): the write pass's bit window (12 / 16 words) and one store
# instruction per flushed block (ICX_DEC_DC_LANE): decode parity with two
# variants, then the e2e A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in w16 dcl; do
  ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_$v.so timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -x -q \
      -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4o.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r4o.log; exit 1; }
done
tail -2 gpurun_out/pytest_gpu_r4o.log
ROUNDS=2 bash scripts/ab_e2e.sh base lib/libicx_w12.so lib/libicx_w16.so lib/libicx_dcl.so 2>&1 | tee gpurun_out/ab_r4o_dec_win.txt
