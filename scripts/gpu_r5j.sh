#!/bin/bash
# Round 5 (j): rocprofv3 kernel statistics of the decoder alone
# (scripts/bench_decode.py, 1000 and 200 4K q95 frames per call), so each
# decode kernel's time can be set against its bytes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
for fr in 1000 200; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_dec$fr" -o run \
      -- python3 "$R/scripts/bench_decode.py" --frames $fr --steps 3 --distinct 16 \
      > "$R/gpurun_out/prof_dec$fr.out" 2>&1 || { echo "rocprof $fr failed"; tail -20 "$R/gpurun_out/prof_dec$fr.out"; exit 1; }
  find "$R/gpurun_out/prof_dec$fr" -name '*kernel_stats.csv' -exec cp {} "$R/gpurun_out/rocprof_r5j_dec${fr}_kernel_stats.csv" \;
  for f in $(find "$R/gpurun_out/prof_dec$fr" -name '*kernel_trace.csv'); do
    { head -1 "$f"; grep -E 'k_dec|k_unstuff|k_stage' "$f" || true; } > "$R/gpurun_out/trace_r5j_dec$fr.csv"
  done
  rm -rf "$R/gpurun_out/prof_dec$fr"
  python3 - "$R/gpurun_out/rocprof_r5j_dec${fr}_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e6:9.3f} ms avg {float(r['TotalDurationNs'])/1e6:9.2f} ms total")
PY
done
