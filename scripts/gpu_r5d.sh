#!/bin/bash
# Round 5 (d): GPU tests (CMYK / YCCK device decode added), decode A/B of
# the 9-bit first level (write pass back to 40 KiB of LDS) and of the sync
# walk's table layout, and the host IO probe of the files -> files path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -s \
    > gpurun_out/pytest_gpu_r5d.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r5d.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r5d.log
echo "== decode A/B 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh lib/libicx_r4.so base lib/libicx_nosplit.so lib/libicx_lut9.so lib/libicx_lut9ns.so || exit 1
echo "== decode A/B 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh lib/libicx_r4.so base lib/libicx_nosplit.so lib/libicx_lut9.so lib/libicx_lut9ns.so ICX_DEC_TAIL_SPLIT=2 || exit 1
echo "== host io"
timeout -k 10 300 python scripts/host_io_probe.py --files 1000 --threads 16 > gpurun_out/host_io_r5d.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/host_io_r5d.log; exit 1; }
cat gpurun_out/host_io_r5d.log | grep -v "^{"
timeout -k 10 300 python scripts/host_io_probe.py --files 1000 --threads 8 > gpurun_out/host_io_r5d_t8.log 2>&1 || exit 1
grep "_r1" gpurun_out/host_io_r5d_t8.log
