#!/bin/bash
# A/B timing of the device JPEG decoder on the GPU box (scripts/bench_decode.py,
# 200 4K q95 frames, mixed content), variants interleaved like scripts/ab.sh:
#   scripts/ab_decode.sh base lib/libicx_x.so ICX_X=1 lib/libicx_y.so:ICX_Y=2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq $ROUNDS); do
  for v in "$@"; do
    lib=image-compression_amd/$v; envs=""
    case "$v" in
      base) lib=image-compression_amd/lib/libicx.so ;;
      *.so:*=*) lib=image-compression_amd/${v%%:*}; envs=${v#*:} ;;  # lib/x.so:ENV=V
      *=*) lib=image-compression_amd/lib/libicx.so; envs=$v ;;
    esac
    env $envs ICX_LIB=$(pwd)/$lib timeout -k 10 180 python scripts/bench_decode.py --frames ${FRAMES:-200} \
        --steps ${STEPS:-5} ${AB_ARGS} > gpurun_out/abd.json 2> gpurun_out/abd.err \
        || { echo "$v failed"; tail -5 gpurun_out/abd.err; exit 1; }
    python3 - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abd.json").read().strip().splitlines()[-1])
k = d["kernels_ms_per_step"]
print(f"{sys.argv[1]:>26s} {d['ms_per_step']:7.2f} ms {d['value']:8.0f} MP/s | " +
      " ".join(f"{n[4:]} {v:.2f}" for n, v in k.items()) + f" | sync x{d['sync_launches_per_step']:.1f}", flush=True)
PY
  done
done
