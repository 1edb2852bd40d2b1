#!/bin/bash
# Round 4, first box: parity tests, the default bench line, the layout-flip count.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4a} SKIP_PROF=1 bash scripts/gpu_round.sh || exit 1
timeout -k 10 300 python scripts/layout_flips.py --gpu > gpurun_out/layout_flips_gpu.json 2> gpurun_out/layout_flips_gpu.err \
    || { echo "layout_flips failed"; tail -20 gpurun_out/layout_flips_gpu.err; exit 1; }
cat gpurun_out/layout_flips_gpu.json
