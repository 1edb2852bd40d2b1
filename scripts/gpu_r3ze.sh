set -o pipefail
ROUNDS=5 timeout -k 10 1000 bash scripts/ab.sh lib/libicx_prev.so base lib/libicx_t3.so lib/libicx_t4.so > gpurun_out/ab_r3ze_fdct_tiles.txt 2>&1 || exit 1
cat gpurun_out/ab_r3ze_fdct_tiles.txt
