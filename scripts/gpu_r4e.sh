#!/bin/bash
# Round 4 (e): relops GPU tests + relops bench under a kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops strings tpch]"
timeout -k 10 400 python -u -m pytest tests/test_relops.py tests/test_strings.py tests/test_tpch.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
echo "[relops trace]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/relops_prof -o run --output-format csv -- python3 scripts/bench_relops.py --rounds 2 > $O/relops_prof.log 2>&1 || { tail -20 $O/relops_prof.log; exit 1; }
echo "[tpch sf1]"
timeout -k 10 400 python -u scripts/bench_tpch.py --sf 1 --rounds 3 --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo done
