#!/bin/bash
# Round 4 (za): files -> files JPEG pipeline, device batch (group) size sweep
# with one and two GPU workers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for dev in 0 0,0; do
  for g in 64 128 250; do
    timeout -k 10 300 python scripts/bench_pipeline.py --files 1000 --devices $dev --group $g > gpurun_out/pipe_za_${dev/,/}_$g.json 2>> gpurun_out/pipe_za.err \
        || { echo "pipeline $dev $g failed"; tail -20 gpurun_out/pipe_za.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['runs'][-1]; print(sys.argv[2], sys.argv[3], r['run'], r['images_per_s'], r['stages']['gpu_decode'])" gpurun_out/pipe_za_${dev/,/}_$g.json $dev $g
  done
done
