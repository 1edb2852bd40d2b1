#!/bin/bash
# Round 5 (b): GPU tests (self-check, icx_upload), then files -> files with
# reader-side uploads (DeviceReader) at group 64 / 128, one and two workers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -s \
    > gpurun_out/pytest_gpu_r5b.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r5b.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r5b.log
grep "icx_create ms" gpurun_out/pytest_gpu_r5b.log
for g in 64 128; do
  for dv in 0 0,0; do
    timeout -k 10 300 python scripts/bench_pipeline.py --files 1000 --group $g --devices $dv > gpurun_out/pipeline_r5b_g${g}_d${dv/,/}.json 2>> gpurun_out/pipeline_r5b.err \
        || { echo "pipeline $g $dv failed"; tail -20 gpurun_out/pipeline_r5b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/pipeline_r5b_g${g}_d${dv/,/}.json')); print('$g $dv', [(r['run'], r['images_per_s'], r['device_busy_frac'], r['stages'].get('gpu_decode'), r['stages'].get('upload')) for r in d['runs']])"
  done
done
