#!/bin/bash
# Round 5 (u): the e2e leg over three contexts at once (bench.py
# e2e.concurrent, the CLI's workers per device) beside the serial one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-io-frames 0 > gpurun_out/bench_r5u.json 2> gpurun_out/bench_r5u.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench_r5u.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r5u.json').read().strip().splitlines()[-1])
e=d['e2e']; print('value', d['value'], 'e2e', e['value'], 'decode', e['decode_mp_s'], 'concurrent', e.get('concurrent'))"
