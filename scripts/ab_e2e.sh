#!/bin/bash
# A/B of libicx variants on bench.py's e2e leg (1000 distinct 4K q95 sources in
# HBM -> decode -> target-size encode, and the 200-frame call), variants
# interleaved: scripts/ab_e2e.sh base lib/libicx_x.so ICX_X=1,ICX_Y=2 lib/libicx_x.so:ICX_X=1
# (NAME=VALUE[,NAME=VALUE]: the default library under those environment
# variables; LIB:NAME=VALUE: that library under them)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq $ROUNDS); do
  for v in "$@"; do
    lib=image-compression_amd/$v; envs=""
    case "$v" in
      base) lib=image-compression_amd/lib/libicx.so ;;
      *.so:*) lib=image-compression_amd/${v%%:*}; envs=${v#*:}; envs=${envs//,/ } ;;
      *=*) lib=image-compression_amd/lib/libicx.so; envs=${v//,/ } ;;
    esac
    env $envs ICX_LIB=$(pwd)/$lib timeout -k 10 240 python bench.py --images 1000 --e2e ${FRAMES:-1000} --steps ${STEPS:-3} \
        --warmup 1 --no-cpu-baseline --host-io-frames 0 --pool-devices none --profile 0 \
        > gpurun_out/abe.json 2> gpurun_out/abe.err || { echo "$v failed"; tail -5 gpurun_out/abe.err; exit 1; }
    python3 - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abe.json").read().strip().splitlines()[-1])["e2e"]
s = d.get("at_small_batch", {})
print(f"{sys.argv[1]:>28s} e2e {d['value']:8.0f} | decode {d['decode_ms_per_step']:7.2f} ms {d['decode_mp_s']:8.0f} MP/s"
      f" | @{s.get('frames')} decode {s.get('decode_ms_per_step', 0):6.2f} ms {s.get('decode_mp_s', 0):8.0f}", flush=True)
PY
  done
done
