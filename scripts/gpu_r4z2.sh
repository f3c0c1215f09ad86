#!/bin/bash
# Round 4 (z2): batch device from string columns too — Q12 path check + TPC-H all ten at SF1 / SF10 checked.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4z2
mkdir -p $O
timeout -k 10 300 python -u scripts/debug_q12_groupby.py > $O/debug.log 2>&1 || { tail -30 $O/debug.log; exit 1; }
grep -v "^$" $O/debug.log | tail -5
timeout -k 10 900 python -u scripts/bench_tpch.py --sf 1,10 --queries q01,q02,q03,q04,q06,q12,q13,q14,q17,q22 --stage-times --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{\"sf\"" $O/tpch.log
echo done
