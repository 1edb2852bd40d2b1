#!/bin/bash
# GPU-box helper for one measurement round: parity tests, the default bench
# line, and a rocprofv3 kernel-trace summary of the headline alone (no e2e
# leg, no CPU baseline: the summary's per-kernel means are the timed region's).
# Every GPU step has its own time limit; the first failure ends the script.
# Knobs (environment): TAG, SKIP_TESTS, PYTEST_ARGS, BENCH_ARGS, SKIP_PROF,
# PROF_ARGS, T_TESTS / T_BENCH / T_PROF, and EXTRA: one more command (an A/B,
# a decode or pipeline bench) run last under its own limit T_EXTRA, its
# output in gpurun_out/extra_${TAG}.log - what the round-by-round one-off
# launchers (git history: scripts/gpu_r*.sh) did.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-r2}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${T_TESTS:-600} python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS} > gpurun_out/pytest_gpu_${TAG}.log 2>&1
  rc=$?
  tail -15 gpurun_out/pytest_gpu_${TAG}.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
timeout -k 10 ${T_BENCH:-400} python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench_${TAG}.json \
    2> gpurun_out/bench_${TAG}.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
if [ -z "$SKIP_PROF" ]; then
  cd /tmp
  timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}" -o run \
      -- python3 "$R/bench.py" ${PROF_ARGS:---steps 20 --warmup 5 --e2e 0 --no-cpu-baseline --host-io-frames 0} \
      > "$R/gpurun_out/prof_${TAG}.out" 2>&1 || { echo "rocprof failed rc=$?"; tail -20 "$R/gpurun_out/prof_${TAG}.out"; exit 1; }
  cd "$R"
  find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' -exec cat {} \;
  grep -h '^{' gpurun_out/prof_${TAG}.out | tail -1 > gpurun_out/prof_${TAG}_bench.json || true
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 ${T_EXTRA:-600} bash -o pipefail -c "$EXTRA" > gpurun_out/extra_${TAG}.log 2>&1 \
      || { echo "extra failed rc=$?"; tail -20 gpurun_out/extra_${TAG}.log; exit 1; }
  tail -20 gpurun_out/extra_${TAG}.log
fi
