#!/bin/bash
# Round 5 (s): lazy byte classification in the unstuffing kernels (only the
# bytes after a 0xFF classified as zero / RSTn) - decode parity on that build,
# decode A/B against the default; then files -> files repeated with the
# inputs' page-cache writeback moved out of the timed runs (os.sync).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe_s
ICX_LIB=$R/image-compression_amd/lib/libicx_lazy.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_decode_gpu.py tests/test_cmyk_gpu.py > gpurun_out/pytest_gpu_r5s.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r5s.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5s.log
echo "== 1000 frames"
FRAMES=1000 STEPS=3 AB_ARGS="--distinct 16" ROUNDS=2 bash scripts/ab_decode.sh base lib/libicx_lazy.so || exit 1
echo "== 200 frames"
FRAMES=200 AB_ARGS="--distinct 16" ROUNDS=1 bash scripts/ab_decode.sh base lib/libicx_lazy.so || exit 1
echo "== files -> files, two workers"
for r in 1 2 3 4; do
  timeout -k 10 240 python scripts/bench_pipeline.py --files 1000 --group 64 --devices 0,0 \
      > gpurun_out/pipe_s/d00_$r.json 2>> gpurun_out/pipe_s/err.log || { echo "run $r failed"; tail -20 gpurun_out/pipe_s/err.log; exit 1; }
  python3 - gpurun_out/pipe_s/d00_$r.json $r <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["runs"][1]
dm = r["device_ms"]
print(f"{sys.argv[2]:>4s} {r['images_per_s']:7.1f} files/s busy {r['device_busy_frac']:.3f} dev {r['device_ms_total']:6.1f} ms "
      f"stage {r['stages']['stage']['seconds']:.2f} write {r['stages']['write']['seconds']:.2f} | learn {d['runs'][0]['images_per_s']:7.1f}", flush=True)
PY
done
