#!/bin/bash
# Round 5 (r): 32768-bit subsequences for 64-frame decode calls (the
# pipeline's group), GPU tests, then files -> files repeated on the default
# CLI layout (two workers), one and three workers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe_r
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_r5r.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r5r.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5r.log
for r in 1 2 3 4; do
  for dv in 0,0 0 0,0,0; do
    [ $r -gt 2 ] && [ $dv != 0,0 ] && continue
    n=d${dv//,/}_$r
    timeout -k 10 240 python scripts/bench_pipeline.py --files 1000 --group 64 --devices $dv \
        > gpurun_out/pipe_r/$n.json 2>> gpurun_out/pipe_r/err.log || { echo "$n failed"; tail -20 gpurun_out/pipe_r/err.log; exit 1; }
    python3 - gpurun_out/pipe_r/$n.json $n <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["runs"][1]
dm = r["device_ms"]
print(f"{sys.argv[2]:>10s} {r['images_per_s']:7.1f} files/s busy {r['device_busy_frac']:.3f} dev {r['device_ms_total']:6.1f} ms "
      f"sync {sum(v for k, v in dm.items() if k.startswith('dec_sync')):6.1f} write {dm.get('dec_write', 0):5.1f} "
      f"| learn {d['runs'][0]['images_per_s']:7.1f}", flush=True)
PY
  done
done
