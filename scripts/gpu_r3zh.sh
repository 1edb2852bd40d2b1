set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r3zh.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3zh.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r3zh.log
# the per-workgroup entry count must credit exactly what the per-wave atomics did
for v in lib/libicx_prev.so lib/libicx.so; do
  ICX_LIB=$(pwd)/image-compression_amd/$v timeout -k 10 180 python bench.py --images 300 --e2e 0 --no-cpu-baseline --host-io-frames 0 --steps 1 --warmup 0 > gpurun_out/ent.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ent.json')); k=d['kernels']; print('$v', 'fdct algo bytes', k['fdct'].get('algo_bytes'), 'huff algo bytes', k['huff'].get('algo_bytes'))"
done
ROUNDS=4 timeout -k 10 900 bash scripts/ab.sh lib/libicx_prev.so lib/libicx_noat.so base > gpurun_out/ab_r3zh_fdct_ent.txt 2>&1 || exit 1
cat gpurun_out/ab_r3zh_fdct_ent.txt
