#!/bin/bash
# Round 5 (t): workers per GPU for files -> files (two = the CLI default;
# three / four contexts overlap more of each other's latency-bound
# relaxation launches), interleaved, page-cache writeback outside the runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe_t
for r in 1 2 3; do
  for dv in 0,0 0,0,0 0,0,0,0; do
    n=d${dv//,/}_$r
    timeout -k 10 240 python scripts/bench_pipeline.py --files 1000 --group 64 --devices $dv \
        > gpurun_out/pipe_t/$n.json 2>> gpurun_out/pipe_t/err.log || { echo "$n failed"; tail -20 gpurun_out/pipe_t/err.log; exit 1; }
    python3 - gpurun_out/pipe_t/$n.json $n <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["runs"][1]
print(f"{sys.argv[2]:>10s} {r['images_per_s']:7.1f} files/s busy {r['device_busy_frac']:.3f} dev {r['device_ms_total']:6.1f} ms "
      f"stage {r['stages']['stage']['seconds']:.2f} write {r['stages']['write']['seconds']:.2f} | learn {d['runs'][0]['images_per_s']:7.1f}", flush=True)
PY
  done
done
