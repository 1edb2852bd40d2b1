set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r3zq.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3zq.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r3zq.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_r3zq_default.json 2> gpurun_out/bench_r3zq.err || { tail -20 gpurun_out/bench_r3zq.err; exit 1; }
cat gpurun_out/bench_r3zq_default.json
