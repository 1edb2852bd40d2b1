#!/bin/bash
# Round 5 close: the driver's own checks on the final tree - GPU tests,
# smoke(), and bench.py with no arguments.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r5final.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5final.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_r5final.json 2> gpurun_out/bench_r5final.err || { tail -20 gpurun_out/bench_r5final.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r5final.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['steps'], d['warmup'], d['roofline']['frac'], d['e2e']['decode_mp_s'], d['cpu_baseline']['value'])"
