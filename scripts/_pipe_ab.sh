set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pipe6b
for cfg in "0,0 64" "0,0 256" "0,0,0 256" "0,0,0,0 256" "0,0,0 512"; do
  set -- $cfg
  tag=$(echo $1 | tr -d ,)_g$2
  timeout -k 10 400 python -u scripts/bench_pipeline.py --files 1000 --devices $1 --group-max $2 --reps 3 > gpurun_out/pipe6b/pipeline_d${tag}.json 2> gpurun_out/pipe6b/pipeline_d${tag}.err || { echo "failed $cfg"; tail -20 gpurun_out/pipe6b/pipeline_d${tag}.err; exit 1; }
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/pipe6b/pipeline_d${tag}.json'))
print('$cfg', json.dumps(d['summary']))"
done
