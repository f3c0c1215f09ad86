#!/bin/bash
# Round 4 (c): string/relops/tpch GPU tests, TPC-H SF1 checked run, rocprof kernel trace of TPC-H SF1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4c
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: strings relops tpch]"
timeout -k 10 400 python -u -m pytest tests/test_strings.py tests/test_relops.py tests/test_tpch.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
tail -5 $O/relops.log
echo "[tpch sf1 checked]"
timeout -k 10 400 python -u scripts/bench_tpch.py --sf ${SF:-1} --rounds 3 --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
cat $O/tpch.log
echo "[tpch trace]"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/tpch_prof -o run --output-format csv -- python3 scripts/bench_tpch.py --sf 1 --rounds 1 --no-check > $O/tpch_prof.log 2>&1 || { tail -20 $O/tpch_prof.log; exit 1; }
echo done
