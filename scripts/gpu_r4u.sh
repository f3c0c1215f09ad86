#!/bin/bash
# Round 4 (u): join-build table preset without a host->device copy; TPC-H SF10 join-heavy queries with stage times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4u
mkdir -p $O
export TMPDIR=/tmp
echo "[tpch]"
timeout -k 10 600 python -u scripts/bench_tpch.py --sf 10 --queries q03,q12,q04,q17,q01 --stage-times --no-check --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo done
