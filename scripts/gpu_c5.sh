#!/bin/bash
# GPU-box helper: parity tests, then the PNG half of configs[4] (C5: batched
# device fit + host PNG write) with its rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-r3}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${T_TESTS:-600} python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS} > gpurun_out/pytest_gpu_${TAG}.log 2>&1
  rc=$?
  tail -15 gpurun_out/pytest_gpu_${TAG}.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
timeout -k 10 300 python scripts/bench_configs.py --only C5 --frames ${FRAMES:-200} > gpurun_out/c5_${TAG}.jsonl \
    2> gpurun_out/c5_${TAG}.err || { echo "c5 failed rc=$?"; tail -20 gpurun_out/c5_${TAG}.err; exit 1; }
cat gpurun_out/c5_${TAG}.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_c5_${TAG}" -o run \
    -- python3 "$R/scripts/bench_configs.py" --only C5 --frames ${FRAMES:-200} > "$R/gpurun_out/prof_c5_${TAG}.out" 2>&1 \
    || { echo "rocprof failed rc=$?"; tail -20 "$R/gpurun_out/prof_c5_${TAG}.out"; exit 1; }
cd "$R"
grep -h 'icx::' gpurun_out/prof_c5_${TAG}/*kernel_stats.csv || true
