#!/bin/bash
# Round 5 (e): files -> files with native staging (icx_stage_files) at group
# 64 / 128, one and two workers; GPU tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r5e}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$T.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$T.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$T.log
fi
for g in ${GROUPS_:-64 128}; do
  for dv in ${DEVS:-0 0,0}; do
    timeout -k 10 300 python scripts/bench_pipeline.py --files 1000 --group $g --devices $dv ${PIPE_ARGS} > gpurun_out/pipeline_${T}_g${g}_d${dv/,/}.json 2>> gpurun_out/pipeline_$T.err \
        || { echo "pipeline $g $dv failed"; tail -20 gpurun_out/pipeline_$T.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/pipeline_${T}_g${g}_d${dv/,/}.json'))
for r in d['runs']:
    print('$g $dv', r['run'], r['images_per_s'], 'busy', r['device_busy_frac'], {k: round(v['seconds'], 3) for k, v in r['stages'].items()})"
  done
done
