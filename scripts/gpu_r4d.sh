#!/bin/bash
# Round 4 (d): relops kernel trace, TPC-H SF1 + SF10 checked, dedup skinny-GEMM A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4d
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: strings relops tpch storage]"
timeout -k 10 400 python -u -m pytest tests/test_strings.py tests/test_relops.py tests/test_tpch.py tests/test_storage.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[relops trace]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/relops_prof -o run --output-format csv -- python3 scripts/bench_relops.py --rounds 3 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
tail -5 $O/relops.log
echo "[tpch sf1,10 checked]"
timeout -k 10 900 python -u scripts/bench_tpch.py --sf 1,10 --rounds 3 --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
cat $O/tpch.log
echo "[dedup gemm ab]"
timeout -k 10 200 python -u scripts/ab_dedup_gemm.py > $O/ab_dedup.log 2>&1 || { tail -20 $O/ab_dedup.log; exit 1; }
cat $O/ab_dedup.log
echo done
