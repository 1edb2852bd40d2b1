#!/bin/bash
# Round 5 (q): files -> files A/B on the default CLI layout (two workers on
# one GPU, group 64): subsequence length of the 64-frame decode calls
# (pick_sub_bits gives 16384 there: four sync launches per call) and group
# size; each setting twice (runs on one box vary by ~10 %).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe_q
# k_huff's per-dispatch fetch: which launches carry the excess (pmc_summary
# r5p: 10 of 12 fetch 0.965x the algorithmic bytes, two 1.39x)
R=$(pwd)
( cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_q" -o run \
    -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --e2e 0 --host-io-frames 0 > "$R/gpurun_out/pmc_q.out" 2>&1 ) \
    || { echo "pmc failed"; tail -20 gpurun_out/pmc_q.out; exit 1; }
for f in $(find gpurun_out/pmc_q -name '*counter_collection.csv'); do
  { head -1 "$f"; grep -E 'k_huff|k_fdct|k_scan|k_stuff' "$f" || true; } > gpurun_out/pmc_q_huff_dispatches.csv
done
for f in $(find gpurun_out/pmc_q -name '*kernel_trace.csv'); do
  { head -1 "$f"; grep -E 'k_huff|k_fdct|k_scan|k_stuff|k_list' "$f" || true; } > gpurun_out/pmc_q_trace.csv
done
rm -rf gpurun_out/pmc_q
run() {  # name env... -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  for r in 1 2; do
    env "${envs[@]}" timeout -k 10 240 python scripts/bench_pipeline.py --files 1000 "$@" \
        > gpurun_out/pipe_q/${name}_$r.json 2>> gpurun_out/pipe_q/err.log \
        || { echo "$name failed"; tail -20 gpurun_out/pipe_q/err.log; return 1; }
    python3 - gpurun_out/pipe_q/${name}_$r.json "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["runs"][1]
dm = r["device_ms"]
print(f"{sys.argv[2]:>22s} {r['images_per_s']:7.1f} files/s busy {r['device_busy_frac']:.3f} dev {r['device_ms_total']:6.1f} ms "
      f"sync {dm.get('dec_sync',0)+dm.get('dec_sync_r1',0)+dm.get('dec_sync_r2',0)+dm.get('dec_sync_r3',0):6.1f} "
      f"write {dm.get('dec_write',0):5.1f} | learn {d['runs'][0]['images_per_s']:7.1f}", flush=True)
PY
  done
}
run base X=1 -- --devices 0,0 --group 64 || exit 1
run sub32k ICX_DEC_SUB_BITS=32768 -- --devices 0,0 --group 64 || exit 1
run sub64k ICX_DEC_SUB_BITS=65536 -- --devices 0,0 --group 64 || exit 1
run g96 X=1 -- --devices 0,0 --group 96 || exit 1
run g128sub32k ICX_DEC_SUB_BITS=32768 -- --devices 0,0 --group 128 || exit 1
