#!/bin/bash
# Round 4 (zh): files -> files JPEG pipeline at configs[1]'s size with the
# round's decoder (one and two GPU workers), and a decode timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/bench_pipeline.py --files 1000 > gpurun_out/pipeline_r4zh_jpeg1000.json 2> gpurun_out/pipeline_r4zh.err \
    || { echo "pipeline failed"; tail -20 gpurun_out/pipeline_r4zh.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/pipeline_r4zh_jpeg1000.json')); print([(r['run'], r['images_per_s']) for r in d['runs']])"
timeout -k 10 400 python scripts/bench_pipeline.py --files 1000 --devices 0,0 > gpurun_out/pipeline_r4zh_jpeg1000_dev00.json 2>> gpurun_out/pipeline_r4zh.err \
    || { echo "pipeline 0,0 failed"; tail -20 gpurun_out/pipeline_r4zh.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/pipeline_r4zh_jpeg1000_dev00.json')); print([(r['run'], r['images_per_s']) for r in d['runs']])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_r4zh" -o run \
    -- python3 "$R/bench.py" --images 1000 --e2e 1000 --steps 2 --warmup 1 --no-cpu-baseline --host-io-frames 0 --profile 0 \
    > "$R/gpurun_out/trace_r4zh.out" 2>&1 || { echo "trace failed"; tail -20 "$R/gpurun_out/trace_r4zh.out"; exit 1; }
cd "$R"
for f in $(find gpurun_out/trace_r4zh -name '*kernel_trace.csv'); do
  { head -1 "$f"; grep -E 'k_dec|k_unstuff|k_stage' "$f" || true; } > gpurun_out/trace_r4zh_dec.csv
  rm -f "$f"
done
python3 scripts/dec_timeline.py gpurun_out/trace_r4zh_dec.csv > gpurun_out/dec_timeline_r4zh.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/dec_timeline_r4zh.json"))
for c in d["calls"]:
    print(c["span_ms"], "pre", c["to_first_sync_ms"], "sync0", c["first_sync_ms"], "relax", c["relaxation_ms"], "tail",
          c["tail_after_last_sync_ms"], {k: v["ms"] for k, v in c["kernels_ms"].items()})
PY
