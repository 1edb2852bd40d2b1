#!/bin/bash
# Round 5 (ac): group size with three workers (the CLI default): 64 / 96 / 128
# JPEGs per device batch, interleaved, two runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe_ac
for r in 1 2; do
  for g in 64 96 128; do
    n=g${g}_$r
    timeout -k 10 240 python scripts/bench_pipeline.py --files 1000 --group $g --devices 0,0,0 \
        > gpurun_out/pipe_ac/$n.json 2>> gpurun_out/pipe_ac/err.log || { echo "$n failed"; tail -20 gpurun_out/pipe_ac/err.log; exit 1; }
    python3 - gpurun_out/pipe_ac/$n.json $n <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["runs"][1]
print(f"{sys.argv[2]:>8s} {r['images_per_s']:7.1f} files/s busy {r['device_busy_frac']:.3f} dev {r['device_ms_total']:6.1f} ms "
      f"| learn {d['runs'][0]['images_per_s']:7.1f}", flush=True)
PY
  done
done
