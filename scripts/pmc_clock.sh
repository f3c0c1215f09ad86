#!/bin/bash
# Sustained clock of the FF layer-1 GEMM: GRBM_GUI_ACTIVE cycles per dispatch vs its kernel-trace duration,
# over 60 back-to-back dispatches (ramp visible), then the same for the FF output-layer GEMM.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R"
mkdir -p gpurun_out/clk
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$R/gpurun_out/clk/l1" -o run \
  -- python3 scripts/prof_gemm.py 1000 1000 597568 2 60 > gpurun_out/clk/l1.log 2>&1 || { tail -20 gpurun_out/clk/l1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$R/gpurun_out/clk/l2" -o run \
  -- python3 scripts/prof_gemm.py 1000 14588 1024 2 60 > gpurun_out/clk/l2.log 2>&1 || { tail -20 gpurun_out/clk/l2.log; exit 1; }
find gpurun_out/clk -name "*.csv" | head -20
