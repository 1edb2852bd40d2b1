#!/bin/bash
# Round 4: parity tests of the tree (wave-chunk k_huff), the default bench line,
# A/B of k_huff designs (ICX_HUFF_WAVE=0: 256-block workgroup chunks), layout flips.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4a} SKIP_PROF=1 bash scripts/gpu_round.sh || exit 1
ROUNDS=3 timeout -k 10 900 bash scripts/ab.sh base lib/libicx_hw0.so > gpurun_out/ab_r4a_huff_wave.txt 2>&1 \
    || { echo "ab failed"; cat gpurun_out/ab_r4a_huff_wave.txt; exit 1; }
cat gpurun_out/ab_r4a_huff_wave.txt
timeout -k 10 300 python scripts/layout_flips.py --gpu > gpurun_out/layout_flips_gpu.json 2> gpurun_out/layout_flips_gpu.err \
    || { echo "layout_flips failed"; tail -20 gpurun_out/layout_flips_gpu.err; exit 1; }
cat gpurun_out/layout_flips_gpu.json
