set -o pipefail
ROUNDS=4 timeout -k 10 900 bash scripts/ab.sh base lib/libicx_t2.so lib/libicx_t4.so lib/libicx_noh.so > gpurun_out/ab_r3zl_fdct_tiles2.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zl_fdct_tiles2.txt
