set -o pipefail
# the k_stuff chunks-per-wave variant (lib/libicx_cpw2.so) through the GPU parity tests, then the A/B
ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_cpw2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r3zm.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3zm.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r3zm.log
ROUNDS=4 timeout -k 10 900 bash scripts/ab.sh base lib/libicx_cpw1.so lib/libicx_cpw2.so lib/libicx_cpw4.so > gpurun_out/ab_r3zm_stuff_cpw.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zm_stuff_cpw.txt
