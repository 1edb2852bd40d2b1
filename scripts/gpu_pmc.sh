#!/bin/bash
# GPU-box helper: HBM traffic per kernel from rocprofv3 PMC counters, one
# counter group per pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE do not
# fit one TCC pass), kernel-trace only alongside.  Config: every trial active
# (no cache, huge target -> 5 search trials all fitting).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-r1}
ARGS=${PMC_ARGS:-"--images 64 --steps 1 --warmup 0 --no-cpu-baseline --profile 0 --no-cache --target 16000000 --e2e 0"}
mkdir -p gpurun_out/pmc_${TAG}
cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${T_PMC:-300} rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_${TAG}/$ctr" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_${TAG}/$ctr.out" 2>&1 || { echo "pmc $ctr failed rc=$?"; tail -20 "$R/gpurun_out/pmc_${TAG}/$ctr.out"; exit 1; }
done
cd "$R"
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG} fdct=$((64*3840*2160)) huff=$((64*194400))
