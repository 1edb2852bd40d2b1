#!/bin/bash
# Round 4 (z): kernel traces of the decode calls with one and two aux (tail)
# streams, per-launch listings of the 200-frame calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
for aux in 1 2; do
  cd /tmp
  ICX_DEC_AUX=$aux timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_r4z_$aux" -o run \
      -- python3 "$R/bench.py" --images 1000 --e2e 1000 --steps 2 --warmup 1 --no-cpu-baseline --host-io-frames 0 --profile 0 --pool-devices none \
      > "$R/gpurun_out/trace_r4z_$aux.out" 2>&1 || { echo "trace failed"; tail -20 "$R/gpurun_out/trace_r4z_$aux.out"; exit 1; }
  cd "$R"
  for f in $(find gpurun_out/trace_r4z_$aux -name '*kernel_trace.csv'); do
    { head -1 "$f"; grep -E 'k_dec|k_unstuff|k_stage' "$f" || true; } > gpurun_out/trace_r4z_${aux}_dec.csv
    rm -f "$f"
  done
  python3 scripts/dec_launches.py gpurun_out/trace_r4z_${aux}_dec.csv 3 4 5 > gpurun_out/launches_r4z_$aux.txt
  grep "^call" gpurun_out/launches_r4z_$aux.txt
done
