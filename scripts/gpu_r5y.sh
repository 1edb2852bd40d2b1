#!/bin/bash
# Round 5 (y): decode by content kind (smooth / noise / mixed, 1000 and 200
# frames): per-kind walk rates, to see whether lanes of smooth images (shorter
# codes: more steps per subsequence) set the walk kernels' tails.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/kind
for fr in 1000 200; do
  for kind in smooth noise mixed; do
    timeout -k 10 300 python scripts/bench_decode.py --frames $fr --steps 3 --distinct 16 --kind $kind > gpurun_out/kind/${kind}_$fr.json 2> gpurun_out/kind/err.log \
        || { echo "$kind $fr failed"; tail -20 gpurun_out/kind/err.log; exit 1; }
    python3 - gpurun_out/kind/${kind}_$fr.json $kind $fr <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels_ms_per_step"]
print(f"{sys.argv[2]:>6s} {sys.argv[3]:>5s} {d['ms_per_step']:7.2f} ms {d['value']:8.0f} MP/s bytes {d['mean_jpeg_bytes']:9d} walks {d['sync_walks_per_step']:9.0f} | " +
      " ".join(f"{n[4:]} {v:.2f}" for n, v in k.items()), flush=True)
PY
  done
done
