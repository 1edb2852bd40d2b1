#!/bin/bash
# GPU-box helper: HBM traffic of the headline's kernels from rocprofv3 PMC
# counters, one counter per pass (MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass), kernel-trace alongside; then the
# FETCH_SIZE calibration of k_huff's gather shape (scripts/calib_fetch.hip).
# The bench command is the headline (1000 4K frames, 333-frame sub-batches)
# run as one step without warm-up, so every icx:: dispatch is a timed one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-r2}
ARGS=${PMC_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline --e2e 0 --host-io-frames 0"}
O=$R/gpurun_out/pmc_${TAG}
mkdir -p $O
cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${T_PMC:-300} rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$O/$ctr" -o run \
      -- python3 "$R/bench.py" $ARGS > "$O/$ctr.out" 2>&1 || { echo "pmc $ctr failed rc=$?"; tail -20 "$O/$ctr.out"; exit 1; }
done
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/calib" -o run \
    -- "$R/image-compression_amd/lib/calib_fetch" > "$O/calib.out" 2>&1 || { echo "calib failed rc=$?"; tail -20 "$O/calib.out"; exit 1; }
cd "$R"
python3 scripts/pmc_summary.py $O $O/FETCH_SIZE.out $ARGS
python3 scripts/calib_summary.py $O/calib $O/calib.out
