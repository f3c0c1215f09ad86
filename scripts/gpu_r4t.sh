#!/bin/bash
# Round 4 (t): one coalesced batch per SF10 lineitem scan; TPC-H all ten at SF1 / SF10 checked, with stage times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4t
mkdir -p $O
export TMPDIR=/tmp
echo "[tpch]"
timeout -k 10 900 python -u scripts/bench_tpch.py --sf 1,10 --queries q01,q02,q03,q04,q06,q12,q13,q14,q17,q22 --stage-times --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo done
