set -o pipefail
ROUNDS=4 timeout -k 10 900 bash scripts/ab.sh lib/libicx_prev.so lib/libicx_divonly.so base lib/libicx_t3.so > gpurun_out/ab_r3zd_fdct_split.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zd_fdct_split.txt
