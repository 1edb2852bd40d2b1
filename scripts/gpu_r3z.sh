set -o pipefail
ROUNDS=3 timeout -k 10 500 bash scripts/ab.sh base lib/libicx_wave.so lib/libicx_wave3.so lib/libicx_wave4.so > gpurun_out/ab_fdct_wave_tiles.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --images 1000 --e2e 1000 --steps 3 --warmup 1 --no-cpu-baseline --host-io-frames 0 > gpurun_out/bench_e2e1000.json 2> gpurun_out/bench_e2e1000.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dect -o dect -- python3 scripts/bench_decode.py --frames 200 --distinct 200 --steps 2 --warmup 1 > gpurun_out/dect.log 2>&1
