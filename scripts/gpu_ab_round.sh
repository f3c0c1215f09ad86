#!/bin/bash
# Kernel A/B session: conv tests + conv A/B, FF-tail A/B on the production kernels, store-pattern microbenchmarks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kernel_tests.log 2>&1
rc=$?; tail -3 gpurun_out/kernel_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_conv_full.py --rounds 3 > gpurun_out/ab_conv_ws.log 2>&1 || { cat gpurun_out/ab_conv_ws.log; exit 1; }
cat gpurun_out/ab_conv_ws.log
timeout -k 10 300 python -u scripts/ab_ff_tail.py --rounds 5 > gpurun_out/ab_ff_tail.log 2>&1 || { cat gpurun_out/ab_ff_tail.log; exit 1; }
cat gpurun_out/ab_ff_tail.log
# the store-pattern microbenchmark is built here from its source (no committed binary)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o scripts/native/store_gemm2 scripts/native/store_gemm2.hip || exit 1
timeout -k 10 60 ./scripts/native/store_gemm2 > gpurun_out/store_gemm2.txt 2>&1 || exit 1
cat gpurun_out/store_gemm2.txt
