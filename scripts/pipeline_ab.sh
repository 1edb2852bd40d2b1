#!/bin/bash
# GPU-box helper: files -> files A/B of worker / group configurations
# (scripts/bench_pipeline.py), interleaved over ROUNDS so the box's drift
# over a call does not pick the winner.  CONFIGS: "devices group_max" pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pipe}
mkdir -p gpurun_out/$TAG
CONFIGS=${CONFIGS:-"0,0:0 0,0,0:0"}
for round in $(seq 1 ${ROUNDS:-2}); do
  for cfg in $CONFIGS; do
    dev=${cfg%%:*}; gm=${cfg##*:}
    tag=$(echo $dev | tr -d ,)_g${gm}_r$round
    timeout -k 10 ${T_RUN:-400} python -u scripts/bench_pipeline.py --files ${FILES:-1000} --devices $dev \
        --group-max $gm --reps ${REPS:-3} > gpurun_out/$TAG/pipeline_d${tag}.json 2> gpurun_out/$TAG/pipeline_d${tag}.err \
        || { echo "failed $cfg"; tail -20 gpurun_out/$TAG/pipeline_d${tag}.err; exit 1; }
    python3 -c "
import json
s = json.load(open('gpurun_out/$TAG/pipeline_d${tag}.json'))['summary']
print('$cfg r$round', {k: (v['images_per_s_median'], v['device_busy_frac_median']) for k, v in s.items()})"
  done
done
