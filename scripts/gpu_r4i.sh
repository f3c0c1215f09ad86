#!/bin/bash
# Round 4 (i): full GPU suite, headline bench, relops bench, TPC-H SF 1 + 10 (checked).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4i
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests]"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[bench]"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
echo "[tpch sf1,10]"
timeout -k 10 900 python -u scripts/bench_tpch.py --sf 1,10 --rounds 3 --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo done
