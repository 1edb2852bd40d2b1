set -o pipefail
# every BASELINE config on one MI355X with the final kernels
timeout -k 10 900 python -u scripts/bench_configs.py > gpurun_out/configs_r3zn.jsonl 2> gpurun_out/configs_r3zn.err || { tail -20 gpurun_out/configs_r3zn.err; exit 1; }
cat gpurun_out/configs_r3zn.jsonl
