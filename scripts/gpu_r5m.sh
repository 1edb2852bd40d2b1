#!/bin/bash
# Round 5 measurement: GPU tests, the default bench line, its rocprofv3
# kernel-trace summary (headline only), files -> files (default CLI layout:
# two workers, group 64; and one worker), and a kernel trace of the e2e
# leg's decode calls (scripts/dec_timeline.py).  TAG names the outputs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
T=${TAG:-r5m}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$T.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$T.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$T.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench_$T.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$T.json').read().strip().splitlines()[-1])
e=d['e2e']; print('value', d['value'], 'ms', d['ms_per_step'], 'huff frac', d['roofline']['frac'], 'e2e', e['value'], 'decode', e['decode_ms_per_step'], e['decode_mp_s'], 'small', e['at_small_batch']['decode_ms_per_step'], e['at_small_batch']['decode_mp_s'])"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$T" -o run \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --e2e 0 --no-cpu-baseline --host-io-frames 0 \
    > "$R/gpurun_out/prof_$T.out" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$T.out"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_$T" -o run \
    -- python3 "$R/bench.py" --images 1000 --e2e 1000 --steps 2 --warmup 1 --no-cpu-baseline --host-io-frames 0 --profile 0 \
    > "$R/gpurun_out/trace_$T.out" 2>&1 || { echo "trace failed"; tail -20 "$R/gpurun_out/trace_$T.out"; exit 1; }
cd "$R"
find gpurun_out/prof_$T -name '*kernel_stats.csv' -exec cp {} gpurun_out/rocprof_${T}_kernel_stats.csv \;
grep -h '^{' gpurun_out/prof_$T.out | tail -1 > gpurun_out/prof_${T}_bench.json || true
for f in $(find gpurun_out/trace_$T -name '*kernel_trace.csv'); do
  { head -1 "$f"; grep -E 'k_dec|k_unstuff|k_stage' "$f" || true; } > gpurun_out/trace_${T}_dec.csv
done
rm -rf gpurun_out/trace_$T gpurun_out/prof_$T
python3 scripts/dec_timeline.py gpurun_out/trace_${T}_dec.csv > gpurun_out/dec_timeline_$T.json
python3 -c "
import json; d=json.load(open('gpurun_out/dec_timeline_$T.json'))
for c in d['calls']:
    print(c['span_ms'], 'busy', c['busy_union_ms'], {k: (v['ms'], v['alone_ms']) for k, v in c['kernels_ms'].items()})"
for dv in ${PIPE_DEVS:-0,0,0 0,0 0}; do
  timeout -k 10 300 python scripts/bench_pipeline.py --files 1000 --group 64 --devices $dv > gpurun_out/pipeline_${T}_d${dv//,/}.json 2>> gpurun_out/pipeline_$T.err \
      || { echo "pipeline $dv failed"; tail -20 gpurun_out/pipeline_$T.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/pipeline_${T}_d${dv//,/}.json'))
for r in d['runs']:
    print('$dv', r['run'], r['images_per_s'], 'busy', r['device_busy_frac'], {k: round(v['seconds'], 3) for k, v in r['stages'].items()})"
done
