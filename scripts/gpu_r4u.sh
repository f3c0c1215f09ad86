#!/bin/bash
# Round 4 (u): join build without any host read (device-guarded CSR runs from a bump counter); TPC-H SF10 join-heavy queries with stage times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4u
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops]"
timeout -k 10 300 python -u -m pytest tests/test_relops.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_relops.log 2>&1 || { tail -60 $O/pytest_relops.log; exit 1; }
tail -2 $O/pytest_relops.log
echo "[tpch]"
timeout -k 10 600 python -u scripts/bench_tpch.py --sf 10 --queries q03,q12,q04,q17,q01 --stage-times --no-check --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo done
