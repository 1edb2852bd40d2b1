#!/bin/bash
# Per-dispatch k_huff durations (in launch order) of a short headline run under
# rocprofv3 --kernel-trace, for each variant given as VAR=VALUE or "base":
#   scripts/huff_trace.sh base ICX_X=1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  envs=""; case "$v" in *=*) envs=$v ;; esac
  O=$R/gpurun_out/htrace_$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
  rm -rf "$O"
  (cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O" -o run \
      -- python3 "$R/bench.py" --images ${IMAGES:-300} --e2e 0 --no-cpu-baseline --host-io-frames 0 \
      --steps 1 --warmup 1 > "$O.out" 2>&1) || { echo "$v failed"; tail -5 "$O.out"; exit 1; }
  python3 - "$O" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "icx::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
out = []
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("icx::", "").replace("void ", "")
    out.append(f"{n[:10]}:{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:.3f}")
print(sys.argv[2], " ".join(out[len(out) // 2:]))
PY
  find "$O" -name '*.csv' -delete
done
