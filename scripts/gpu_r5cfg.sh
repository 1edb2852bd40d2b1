#!/bin/bash
# Round 5: every BASELINE config on one MI355X on the final tree
# (scripts/bench_configs.py, inputs and outputs in HBM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/bench_configs.py > gpurun_out/configs_r5.jsonl 2> gpurun_out/configs_r5.err || { tail -20 gpurun_out/configs_r5.err; exit 1; }
cat gpurun_out/configs_r5.jsonl | cut -c1-400
