#!/bin/bash
# Round 4 (c): the files -> files JPEG pipeline with pinned outputs and host
# spans, one GPU worker and two (two contexts on the GPU), then parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/bench_pipeline.py --files 1000 > gpurun_out/pipeline_r4c_jpeg1000.json 2> gpurun_out/pipeline_r4c.err \
    || { echo "pipeline failed"; tail -20 gpurun_out/pipeline_r4c.err; exit 1; }
cat gpurun_out/pipeline_r4c_jpeg1000.json
timeout -k 10 400 python scripts/bench_pipeline.py --files 1000 --devices 0,0 > gpurun_out/pipeline_r4c_jpeg1000_dev00.json 2>> gpurun_out/pipeline_r4c.err \
    || { echo "pipeline 0,0 failed"; tail -20 gpurun_out/pipeline_r4c.err; exit 1; }
cat gpurun_out/pipeline_r4c_jpeg1000_dev00.json
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "pipeline or pool or png or palette" \
    > gpurun_out/pytest_gpu_r4c.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r4c.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r4c.log
