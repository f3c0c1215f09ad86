#!/bin/bash
# Round 4 (o): MID group-by path + exact short-string keys — relops/string tests, relops bench + trace, TPC-H SF1/SF10
# (all ten queries, checked) + a kernel trace of Q01/Q12 at SF10, then the full GPU suite, smoke and the headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4o
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops strings]"
timeout -k 10 300 python -u -m pytest tests/test_relops.py tests/test_strings.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_relops.log 2>&1 || { tail -60 $O/pytest_relops.log; exit 1; }
tail -2 $O/pytest_relops.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_10000 -o run --output-format csv -- python3 scripts/prof_relops_case.py 10000 3 > $O/kt_10000.log 2>&1 || { tail -5 $O/kt_10000.log; exit 1; }
echo "[tpch]"
timeout -k 10 600 python -u scripts/bench_tpch.py --sf 1,10 --queries q01,q02,q03,q04,q06,q12,q13,q14,q17,q22 --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_tpch -o run --output-format csv -- python3 scripts/bench_tpch.py --sf 10 --queries q01,q12 --rounds 1 --no-check > $O/kt_tpch.log 2>&1 || { tail -5 $O/kt_tpch.log; exit 1; }
echo "[gpu suite]"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[smoke]"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[bench]"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log
echo done
