#!/bin/bash
# Fused softmax GEMM study: phase stamps (cold / hot), isolated FF-tail A/B, and the single-job bench under a
# kernel trace. Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/sm
timeout -k 10 180 python scripts/prof_softmax_stamps.py > gpurun_out/sm/stamps.json 2> gpurun_out/sm/stamps.err || { tail -20 gpurun_out/sm/stamps.err; exit 1; }
timeout -k 10 180 python scripts/ab_ff_tail.py > gpurun_out/sm/ab_ff_tail.log 2>&1 || { tail -20 gpurun_out/sm/ab_ff_tail.log; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/sm/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 10 --single-job > gpurun_out/sm/prof.log 2>&1 || { tail -20 gpurun_out/sm/prof.log; exit 1; }
python3 scripts/last_steps.py gpurun_out/sm/prof/run_kernel_trace.csv 12 > gpurun_out/sm/last_steps.txt
cat gpurun_out/sm/stamps.json gpurun_out/sm/ab_ff_tail.log gpurun_out/sm/last_steps.txt
