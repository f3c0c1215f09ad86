#!/bin/bash
# Round 4 (j): relops tests + bench + traces, TPC-H all ten queries at SF 1 and SF 10 (checked).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4j
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops tpch strings]"
timeout -k 10 300 python -u -m pytest tests/test_relops.py tests/test_tpch.py tests/test_strings.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
for d in 8 10000 10000000; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$d -o run --output-format csv -- python3 scripts/prof_relops_case.py $d 3 > $O/kt_$d.log 2>&1 || { tail -5 $O/kt_$d.log; exit 1; }
done
echo "[tpch all queries sf1,10]"
timeout -k 10 1000 python -u scripts/bench_tpch.py --sf 1,10 --rounds 3 --queries q01,q02,q03,q04,q06,q12,q13,q14,q17,q22 --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo done
