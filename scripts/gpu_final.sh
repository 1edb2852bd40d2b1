#!/bin/bash
# GPU-box helper for a round's final measurements of one tree: parity tests,
# the default bench line, a rocprofv3 kernel-trace summary of the headline
# alone, the HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per
# pass) and the SQ issue counters of the headline (two counter groups), all
# of the same command.  Every GPU step has its own time limit; the first
# failure ends the script.  Summaries: scripts/pmc_summary.py, sq_issue.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-final}
# traces and per-dispatch counter rows are reduced to what the summaries read
# (the merged gpurun_out/ must stay under 64 MiB)
slim() {
  find "$1" -name '*kernel_trace.csv' -delete
  for f in $(find "$1" -name '*counter_collection.csv'); do
    { head -1 "$f"; grep 'icx::' "$f" || true; } > "$f.tmp" && mv "$f.tmp" "$f"
  done
}
if [ -z "$SKIP_ROUND" ]; then
  TAG=$TAG bash scripts/gpu_round.sh || exit 1
  slim gpurun_out/prof_${TAG}
fi
ONE="--steps 1 --warmup 0 --no-cpu-baseline --e2e 0 --host-io-frames 0"
O=$R/gpurun_out/pmc_${TAG}
mkdir -p $O
cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$O/$ctr" -o run \
      -- python3 "$R/bench.py" $ONE > "$O/$ctr.out" 2>&1 || { echo "pmc $ctr failed rc=$?"; tail -20 "$O/$ctr.out"; exit 1; }
done
slim "$O"
cd "$R"
TAG=sq_${TAG} SQ_ARGS="$ONE" bash scripts/gpu_sq.sh > gpurun_out/sq_${TAG}.txt 2>&1 || { echo "sq failed"; tail -20 gpurun_out/sq_${TAG}.txt; exit 1; }
slim gpurun_out/sq_${TAG}
du -sh gpurun_out
echo done
