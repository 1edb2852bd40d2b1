set -o pipefail
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_z16.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "huff or parity or encode or golden or fit" > gpurun_out/pytest_gpu_r3zp.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3zp.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r3zp.log
ROUNDS=4 timeout -k 10 900 bash scripts/ab.sh base lib/libicx_z16.so > gpurun_out/ab_r3zp_huff_zero16.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zp_huff_zero16.txt
