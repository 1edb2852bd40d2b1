#!/bin/bash
# GPU-box helper: bench.py (JSON line) + rocprofv3 kernel-trace stats of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r1}
timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
if [ -n "$PROF" ]; then
  cd /tmp
  timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}" -o run -- python3 "$R/bench.py" ${PROF_ARGS} > "$R/gpurun_out/prof_${TAG}.out" 2>&1 || { echo "rocprof failed rc=$?"; tail -20 "$R/gpurun_out/prof_${TAG}.out"; exit 1; }
  cd "$R"
  find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' -exec cat {} \;
fi
