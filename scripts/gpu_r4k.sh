#!/bin/bash
# Round 4 (j): decode parity (subsequence lengths), the e2e leg and
# the decode timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "decode or pipeline or configs" \
    > gpurun_out/pytest_gpu_r4k.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r4k.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r4k.log
timeout -k 10 300 python bench.py --images 1000 --e2e 1000 --steps 5 --warmup 1 --no-cpu-baseline --host-io-frames 0 \
    > gpurun_out/bench_r4k_e2e.json 2> gpurun_out/bench_r4k_e2e.err || { echo "bench failed"; tail -20 gpurun_out/bench_r4k_e2e.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r4k_e2e.json').read().strip().splitlines()[-1]); print(json.dumps(d['e2e']))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_r4k" -o run \
    -- python3 "$R/bench.py" --images 1000 --e2e 1000 --steps 2 --warmup 1 --no-cpu-baseline --host-io-frames 0 --profile 0 \
    > "$R/gpurun_out/trace_r4k.out" 2>&1 || { echo "trace failed"; tail -20 "$R/gpurun_out/trace_r4k.out"; exit 1; }
cd "$R"
for f in $(find gpurun_out/trace_r4k -name '*kernel_trace.csv'); do
  { head -1 "$f"; grep -E 'k_dec|k_unstuff|k_stage' "$f" || true; } > gpurun_out/trace_r4k_dec.csv
  rm -f "$f"
done
python3 scripts/dec_timeline.py gpurun_out/trace_r4k_dec.csv > gpurun_out/dec_timeline_r4k.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/dec_timeline_r4k.json"))
for c in d["calls"]:
    print(c["span_ms"], "pre", c["to_first_sync_ms"], "sync0", c["first_sync_ms"], "relax", c["relaxation_ms"], "tail",
          c["tail_after_last_sync_ms"], {k: v["ms"] for k, v in c["kernels_ms"].items()})
PY
