#!/bin/bash
# asm-scheduled 4-wave GEMM: correctness + interleaved A/B vs the 8-phase kernel, then the GPU test suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
echo "[w4a] check + A/B"
timeout -k 10 300 python -u scripts/ab_w4a.py --rounds ${ROUNDS:-5} ${ABARGS:-} > gpurun_out/ab_w4a.log 2>&1
rc=$?; cat gpurun_out/ab_w4a.log | tail -20; [ $rc -ne 0 ] && exit $rc
if [ "${TESTS:-1}" = "1" ]; then
  echo "[w4a] gpu tests"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu.log; exit $rc
fi
