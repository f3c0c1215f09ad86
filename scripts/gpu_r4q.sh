#!/bin/bash
# Round 4 (q): MID path with its dictionary build in a kernel of its own; one-row shuffle pack fix; two-rank TPC-H
# test; TPC-H SF1/SF10; full suite; smoke; headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4q
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops]"
timeout -k 10 300 python -u -m pytest tests/test_relops.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_relops.log 2>&1 || { tail -60 $O/pytest_relops.log; exit 1; }
tail -2 $O/pytest_relops.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_mid -o run --output-format csv -- python3 scripts/prof_relops_case.py 10000 3 16000000 1 nofirst > $O/kt_mid.log 2>&1 || { tail -5 $O/kt_mid.log; exit 1; }
echo "[two-rank test]"
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1 || { grep -v "^E  *$" $O/pytest_dist.log | grep -A40 "rank failures" | head -80; exit 1; }
tail -2 $O/pytest_dist.log
echo "[tpch]"
timeout -k 10 600 python -u scripts/bench_tpch.py --sf 1,10 --queries q01,q02,q03,q04,q06,q12,q13,q14,q17,q22 --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_tpch -o run --output-format csv -- python3 scripts/bench_tpch.py --sf 10 --queries q01,q12,q03 --rounds 1 --no-check > $O/kt_tpch.log 2>&1 || { tail -5 $O/kt_tpch.log; exit 1; }
echo "[gpu suite]"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_distributed_gpu.py::test_tpch_two_ranks_on_one_gpu_vs_pandas > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[smoke]"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[bench]"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log
echo done
