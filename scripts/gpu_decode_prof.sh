#!/bin/bash
# GPU-box helper: the decoder's own profile - a rocprofv3 kernel trace of
# scripts/bench_decode.py (1000 and 200 frames, 16 distinct sources) reduced
# by scripts/dec_timeline.py, and the SQ counters of a 200-frame call
# (scripts/gpu_sq.sh with SQ_PROG=bench_decode.py).  TAG names the outputs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-dec}
mkdir -p gpurun_out
cd /tmp
for fr in 1000 200; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tl_${TAG}_$fr" -o run \
      -- python3 "$R/scripts/bench_decode.py" --frames $fr --distinct 16 --steps 3 --warmup 1 \
      > "$R/gpurun_out/tl_${TAG}_$fr.out" 2>&1 || { echo "trace $fr failed"; tail -20 "$R/gpurun_out/tl_${TAG}_$fr.out"; exit 1; }
  python3 "$R/scripts/dec_timeline.py" $(find "$R/gpurun_out/tl_${TAG}_$fr" -name '*kernel_trace.csv') \
      > "$R/gpurun_out/dec_timeline_${TAG}_$fr.json" || exit 1
  find "$R/gpurun_out/tl_${TAG}_$fr" -name '*kernel_trace.csv' -delete
done
cd "$R"
TAG=sq_dec_${TAG} SQ_PROG=scripts/bench_decode.py SQ_ARGS="--frames 200 --distinct 16 --steps 1 --warmup 0" \
    bash scripts/gpu_sq.sh > gpurun_out/sq_dec_${TAG}.txt 2>&1 || { echo "sq failed"; tail -20 gpurun_out/sq_dec_${TAG}.txt; exit 1; }
find gpurun_out/sq_dec_${TAG} -name '*kernel_trace.csv' -delete
echo done
