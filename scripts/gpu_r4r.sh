#!/bin/bash
# Round 4 (r): MID path with non-temporal row streams and 64 dictionary-build workgroups; join build fast path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4r
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops]"
timeout -k 10 300 python -u -m pytest tests/test_relops.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_relops.log 2>&1 || { tail -60 $O/pytest_relops.log; exit 1; }
tail -2 $O/pytest_relops.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_mid -o run --output-format csv -- python3 scripts/prof_relops_case.py 10000 3 16000000 1 > $O/kt_mid.log 2>&1 || { tail -5 $O/kt_mid.log; exit 1; }
echo "[tpch sf10]"
timeout -k 10 600 python -u scripts/bench_tpch.py --sf 10 --queries q01,q03,q04,q12,q13,q17 --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo done
