#!/bin/bash
# GPU-box helper: files -> files A/B of library environment settings
# (scripts/bench_pipeline.py, CLI defaults), interleaved over ROUNDS.
#   VARIANTS="base ICX_STAGE_MAP=1" bash scripts/pipeline_env_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pipe_env}
mkdir -p gpurun_out/$TAG
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    envs=""; [ "$v" != base ] && envs=${v//,/ }
    tag=$(echo $v | tr -c 'A-Za-z0-9\n' _)_r$round
    env $envs timeout -k 10 ${T_RUN:-400} python -u scripts/bench_pipeline.py --files ${FILES:-1000} --reps ${REPS:-3} \
        > gpurun_out/$TAG/pipeline_${tag}.json 2> gpurun_out/$TAG/pipeline_${tag}.err \
        || { echo "failed $v"; tail -20 gpurun_out/$TAG/pipeline_${tag}.err; exit 1; }
    python3 -c "
import json
s = json.load(open('gpurun_out/$TAG/pipeline_${tag}.json'))
r = s['runs'][-1]
print('$v r$round', {k: (v['images_per_s_median'], v['device_busy_frac_median']) for k, v in s['summary'].items()},
      'stage thread-s', r['stages']['stage']['seconds'], 'read GB/s', r.get('file_read_GBps'))"
  done
done
