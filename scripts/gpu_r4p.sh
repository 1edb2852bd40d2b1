#!/bin/bash
# Round 4 (p): chroma IDCT with one thread per block in registers
# (ICX_DEC_IDCT_REG): decode parity with it, then the e2e A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ir; do
  ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_$v.so timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -x -q \
      -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4p.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r4p.log; exit 1; }
done
tail -2 gpurun_out/pytest_gpu_r4p.log
ROUNDS=2 bash scripts/ab_e2e.sh base lib/libicx_ir.so 2>&1 | tee gpurun_out/ab_r4p_dec_win.txt
