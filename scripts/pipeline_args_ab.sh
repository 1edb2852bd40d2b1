#!/bin/bash
# GPU-box helper: files -> files A/B of bench_pipeline.py argument sets,
# interleaved over ROUNDS.  VARIANTS: argument sets separated by ';'.
#   VARIANTS="--write-threads 4;--write-threads 16" bash scripts/pipeline_args_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pipe_args}
mkdir -p gpurun_out/$TAG
IFS=';' read -ra SETS <<< "${VARIANTS:-}"
for round in $(seq 1 ${ROUNDS:-2}); do
  k=0
  for v in "${SETS[@]}"; do
    k=$((k+1)); tag=v${k}_r$round
    timeout -k 10 ${T_RUN:-400} python -u scripts/bench_pipeline.py --files ${FILES:-1000} --reps ${REPS:-3} $v \
        > gpurun_out/$TAG/pipeline_${tag}.json 2> gpurun_out/$TAG/pipeline_${tag}.err \
        || { echo "failed $v"; tail -20 gpurun_out/$TAG/pipeline_${tag}.err; exit 1; }
    python3 -c "
import json
s = json.load(open('gpurun_out/$TAG/pipeline_${tag}.json'))
r = s['runs'][-1]
print('$v r$round', {k: (v['images_per_s_median'], v['device_busy_frac_median']) for k, v in s['summary'].items()},
      'stage', r['stages']['stage']['seconds'], 'write', r['stages'].get('write', {}).get('seconds'), 'read GB/s', r.get('file_read_GBps'))"
  done
done
