#!/bin/bash
# Direct-store epilogue validation + A/B: GPU test suite, cfg 2 (transposed acc, direct stores) vs cfg 15
# (LDS-staged store) correctness and timings on the FF layer shapes, GEMM2 epilogue breakdown, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 120 python -u scripts/ab_w4.py --check-only --cfgs 2,15 --shapes 777x555x4104,1000x14588x1000,300x2000x100000 > gpurun_out/store_check.log 2>&1 || exit 1
cat gpurun_out/store_check.log | grep shape
timeout -k 10 200 python -u scripts/ab_w4.py --cfgs 2,15 --rounds 5 --shapes 1000x1000x597568,1000x14588x1000,8192x8192x8192 > gpurun_out/store_ab.log 2>&1 || exit 1
grep ms_min gpurun_out/store_ab.log
timeout -k 10 100 python -u scripts/ab_gemm2_epi.py --cfg 2 > gpurun_out/g2epi_ts.log 2>&1 || exit 1
timeout -k 10 100 python -u scripts/ab_gemm2_epi.py --cfg 15 >> gpurun_out/g2epi_ts.log 2>&1 || exit 1
cat gpurun_out/g2epi_ts.log | grep shape
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
