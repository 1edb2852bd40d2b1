#!/bin/bash
# Round 4 (d): pipeline with pinned slabs + no header re-parse (1 and 2
# workers), and a kernel-trace timeline of the 1000-frame decode calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/bench_pipeline.py --files 1000 > gpurun_out/pipeline_r4d_jpeg1000.json 2> gpurun_out/pipeline_r4d.err \
    || { echo "pipeline failed"; tail -20 gpurun_out/pipeline_r4d.err; exit 1; }
cut -c1-1500 gpurun_out/pipeline_r4d_jpeg1000.json
timeout -k 10 400 python scripts/bench_pipeline.py --files 1000 --devices 0,0 > gpurun_out/pipeline_r4d_jpeg1000_dev00.json 2>> gpurun_out/pipeline_r4d.err \
    || { echo "pipeline 0,0 failed"; tail -20 gpurun_out/pipeline_r4d.err; exit 1; }
cut -c1-1500 gpurun_out/pipeline_r4d_jpeg1000_dev00.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_r4d" -o run \
    -- python3 "$R/bench.py" --images 1000 --e2e 1000 --steps 2 --warmup 1 --no-cpu-baseline --host-io-frames 0 --profile 0 \
    > "$R/gpurun_out/trace_r4d.out" 2>&1 || { echo "trace failed"; tail -20 "$R/gpurun_out/trace_r4d.out"; exit 1; }
cd "$R"
for f in $(find gpurun_out/trace_r4d -name '*kernel_trace.csv'); do
  { head -1 "$f"; grep -E 'k_dec|k_unstuff|k_stage' "$f" || true; } > gpurun_out/trace_r4d_dec.csv
  rm -f "$f"
done
python3 scripts/dec_timeline.py gpurun_out/trace_r4d_dec.csv > gpurun_out/dec_timeline_r4d.json
head -c 3000 gpurun_out/dec_timeline_r4d.json
