#!/bin/bash
# Round 4 (k): relops tests + bench, headline bench (driver args) and its kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops]"
timeout -k 10 300 python -u -m pytest tests/test_relops.py tests/test_tpch.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
for d in 10000 10000000; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$d -o run --output-format csv -- python3 scripts/prof_relops_case.py $d 3 > $O/kt_$d.log 2>&1 || { tail -5 $O/kt_$d.log; exit 1; }
done
echo done
