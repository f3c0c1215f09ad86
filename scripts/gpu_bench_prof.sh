#!/bin/bash
# 1-GPU bench + rocprofv3 kernel trace of the same bench (no test suite).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps ${STEPS:-50} --warmup ${WARMUP:-10} $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 10 $BENCH_ARGS > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
python3 scripts/last_steps.py gpurun_out/prof/run_kernel_trace.csv 15
