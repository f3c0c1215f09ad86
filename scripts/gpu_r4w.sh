#!/bin/bash
# Round 4 (w): join runs fix + planner materialising probe-then-build pipelines — relops tests, TPC-H all ten at
# SF1 / SF10 checked against pandas (stage times), Q03 kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4w
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops tpch]"
timeout -k 10 400 python -u -m pytest tests/test_relops.py tests/test_tpch.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_relops.log 2>&1 || { tail -60 $O/pytest_relops.log; exit 1; }
tail -2 $O/pytest_relops.log
echo "[tpch]"
timeout -k 10 900 python -u scripts/bench_tpch.py --sf 1,10 --queries q01,q02,q03,q04,q06,q12,q13,q14,q17,q22 --stage-times --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_q03 -o run --output-format csv -- python3 scripts/bench_tpch.py --sf 10 --queries q03 --rounds 1 --no-check > $O/kt_q03.log 2>&1 || { tail -5 $O/kt_q03.log; exit 1; }
echo done
