#!/bin/bash
# Round 5 (ar): HBM traffic (PMC FETCH_SIZE / WRITE_SIZE) and SQ issue
# counters of the headline on this round's tree (ICX_COMMIT), and the SQ
# counters of a 200-frame decode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r5ar bash scripts/gpu_pmc.sh > gpurun_out/pmc_r5ar.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_r5ar.log; exit 1; }
rm -rf gpurun_out/pmc_r5ar/FETCH_SIZE gpurun_out/pmc_r5ar/WRITE_SIZE gpurun_out/pmc_r5ar/calib  # raw traces: over gpurun's 64 MiB
grep -A3 '"icx::k_huff"' gpurun_out/pmc_r5ar/pmc_summary.json | head -5
python3 -c "import json; d=json.load(open('gpurun_out/pmc_r5ar/pmc_summary.json')); print(d['tree_commit'], d['bytes_per_unit'], {k: v.get('traffic_over_algo') for k, v in d['kernels'].items()})"
TAG=sq_r5ar SQ_ARGS="--steps 1 --warmup 0 --no-cpu-baseline --e2e 0 --host-io-frames 0" bash scripts/gpu_sq.sh > gpurun_out/sq_r5ar.log 2>&1 || { echo "sq failed"; tail -20 gpurun_out/sq_r5ar.log; exit 1; }
grep -h '^{' gpurun_out/sq_r5ar/libicx.g1.out | tail -1 > gpurun_out/sq_r5ar_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/sq_r5ar_bench.json')); print(d['kernels']['huff']['units'])" > gpurun_out/sq_r5ar_huff_units.txt
python3 scripts/sq_issue.py gpurun_out/sq_r5ar 1000 $(cat gpurun_out/sq_r5ar_huff_units.txt) > gpurun_out/sq_issue_summary_r5ar.json || exit 1
cat gpurun_out/sq_issue_summary_r5ar.json
rm -rf gpurun_out/sq_r5ar/libicx
TAG=sq_r5ar_dec SQ_PROG=scripts/bench_decode.py SQ_ARGS="--frames 200 --steps 1 --warmup 0 --distinct 16" bash scripts/gpu_sq.sh > gpurun_out/sq_r5ar_dec.log 2>&1 || { echo "sq decode failed"; tail -20 gpurun_out/sq_r5ar_dec.log; exit 1; }
rm -rf gpurun_out/sq_r5ar_dec/libicx
tail -60 gpurun_out/sq_r5ar_dec.log | head -5
