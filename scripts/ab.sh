#!/bin/bash
# A/B timing on the GPU box: the headline (one 333-frame sub-batch per step,
# HIP-event kernel times) for each prebuilt library variant, interleaved
# A B A B ... so that drift hits every variant alike.
#   scripts/ab.sh base lib/libicx_x.so ICX_X=1 ...   ("base" = lib/libicx.so;
#   VAR=VALUE = lib/libicx.so with that environment variable)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq $ROUNDS); do
  for v in "$@"; do
    lib=image-compression_amd/$v; envs=""
    case "$v" in base) lib=image-compression_amd/lib/libicx.so ;; *=*) lib=image-compression_amd/lib/libicx.so; envs=$v ;; esac
    env $envs ICX_LIB=$(pwd)/$lib timeout -k 10 180 python bench.py --images ${IMAGES:-300} --e2e 0 --no-cpu-baseline \
        --host-io-frames 0 --steps ${STEPS:-10} --warmup 2 ${AB_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err \
        || { echo "$v failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 - "$v" <<'PY'
import json, sys
d = json.load(open("gpurun_out/ab.json"))
k = d["kernels"]
st = d["steps"]
tot = lambda n: k[n]["ms"] / st if n in k else 0.0
print(f"{sys.argv[1]:>28s} step {d['ms_per_step']:7.3f} ms | per step: fdct {tot('fdct'):.3f} huff {tot('huff'):.3f} "
      f"stuff {tot('stuff'):.3f} scan {tot('scan'):.3f} | huff launches/step {k['huff']['launches'] // st}  "
      f"MP/s {d['value']:.0f}", flush=True)
PY
  done
done
