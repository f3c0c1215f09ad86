#!/bin/bash
# Warp-specialised conv2d: correctness tests, then the isolated A/B vs the full-row / two-pass kernels and MIOpen.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "conv2d" -x -v --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1
rc=$?; tail -4 gpurun_out/conv_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_conv_full.py --rounds 5 > gpurun_out/ab_conv_ws.log 2>&1
rc=$?; cat gpurun_out/ab_conv_ws.log; exit $rc
