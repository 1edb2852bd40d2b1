#!/bin/bash
# GPU-box helper for a measurement round: parity tests, the default bench
# line, the files -> files pipeline over the configs[4] mix (JPEG + PNG,
# warm cache), and the PNG half's batched fit (C5).  Every GPU step has its
# own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_${TAG}.log
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench_${TAG}.json \
    2> gpurun_out/bench_${TAG}.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
if [ -n "$PIPE" ]; then
  timeout -k 10 500 python -u scripts/bench_pipeline.py --files ${PIPE_FILES:-200} --png ${PIPE_PNG:-200} \
      > gpurun_out/pipeline_${TAG}.json 2> gpurun_out/pipeline_${TAG}.err \
      || { echo "pipeline failed rc=$?"; tail -20 gpurun_out/pipeline_${TAG}.err; exit 1; }
  cat gpurun_out/pipeline_${TAG}.json
fi
