#!/bin/bash
# Decode bench at several ICX_DEC_CHECK values (sync launches per host check;
# a large value = no early tails on the aux stream, so the relaunch times are
# free of contention).  Prints ms/step, per-kernel HIP-event ms and relaunch ms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${CHECKS:-2 100}; do
  ICX_DEC_CHECK=$v timeout -k 10 200 python scripts/bench_decode.py --frames 200 --distinct ${DISTINCT:-40} --steps 5 \
      > gpurun_out/dchk_$v.json 2> gpurun_out/dchk_$v.err || { echo "check $v failed"; tail -5 gpurun_out/dchk_$v.err; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/dchk_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], json.dumps(d["kernels_ms_per_step"]), json.dumps(d["sync_relaunch_ms"]),
      d["sync_walks_per_step"], flush=True)
PY
done
