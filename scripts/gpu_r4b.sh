#!/bin/bash
# Round 4 (b): parity tests, the default bench line (host_io / pool / e2e legs),
# the torchrun launch line at nproc 1, the files -> files JPEG pipeline (one
# and two processes), and a kernel trace of the decode + encode leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r4b SKIP_PROF=1 bash scripts/gpu_round.sh || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 1 --steps 3 --warmup 1 --host-io-frames 200 --e2e 200 --no-cpu-baseline \
    > gpurun_out/bench_r4b_torchrun1.json 2> gpurun_out/bench_r4b_torchrun1.err || { echo "torchrun failed"; tail -20 gpurun_out/bench_r4b_torchrun1.err; exit 1; }
tail -c 600 gpurun_out/bench_r4b_torchrun1.json
timeout -k 10 400 python scripts/bench_pipeline.py --files 1000 > gpurun_out/pipeline_r4b_jpeg1000.json 2> gpurun_out/pipeline_r4b.err \
    || { echo "pipeline failed"; tail -20 gpurun_out/pipeline_r4b.err; exit 1; }
cat gpurun_out/pipeline_r4b_jpeg1000.json
timeout -k 10 400 python scripts/bench_pipeline.py --files 1000 --procs 2 > gpurun_out/pipeline_r4b_jpeg1000_2proc.json 2>> gpurun_out/pipeline_r4b.err \
    || { echo "pipeline 2 procs failed"; tail -20 gpurun_out/pipeline_r4b.err; exit 1; }
cat gpurun_out/pipeline_r4b_jpeg1000_2proc.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r4b_e2e" -o run \
    -- python3 "$R/bench.py" --images 1000 --e2e 1000 --steps 2 --warmup 1 --no-cpu-baseline --host-io-frames 0 \
    > "$R/gpurun_out/prof_r4b_e2e.out" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_r4b_e2e.out"; exit 1; }
cd "$R"
find gpurun_out/prof_r4b_e2e -name '*kernel_trace.csv' -delete
find gpurun_out/prof_r4b_e2e -name '*kernel_stats.csv' -exec cat {} \;
