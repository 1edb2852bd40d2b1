#!/bin/bash
# Round 5 (c): GPU tests (self-check, icx_upload, symbol-pair decode), decode
# A/B of the symbol pairs (r4 build, pair builds by write-pass workgroup size
# and sync table layout), then files -> files with reader-side uploads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -s \
    > gpurun_out/pytest_gpu_r5c.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r5c.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r5c.log
grep "icx_create ms" gpurun_out/pytest_gpu_r5c.log
echo "== decode A/B 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh lib/libicx_r4.so base ICX_DEC_PAIR=0 lib/libicx_nt448.so lib/libicx_nt192.so lib/libicx_nosplit.so || exit 1
echo "== decode A/B 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh lib/libicx_r4.so base lib/libicx_nt448.so lib/libicx_nt192.so ICX_DEC_TAIL_SPLIT=2 ICX_DEC_TAIL_SPLIT=3 || exit 1
for g in 64 128; do
  for dv in 0 0,0; do
    timeout -k 10 300 python scripts/bench_pipeline.py --files 1000 --group $g --devices $dv > gpurun_out/pipeline_r5c_g${g}_d${dv/,/}.json 2>> gpurun_out/pipeline_r5c.err \
        || { echo "pipeline $g $dv failed"; tail -20 gpurun_out/pipeline_r5c.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/pipeline_r5c_g${g}_d${dv/,/}.json')); print('$g $dv', [(r['run'], r['images_per_s'], r['device_busy_frac'], r['stages'].get('gpu_decode'), r['stages'].get('upload')) for r in d['runs']])"
  done
done
