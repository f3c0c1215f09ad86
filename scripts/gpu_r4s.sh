#!/bin/bash
# Round 4 (s): TPC-H SF10 per-stage device times (stage-synced extra run per query), relops bench (MID opt-in).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4s
mkdir -p $O
export TMPDIR=/tmp
echo "[tpch sf10 stage times]"
timeout -k 10 600 python -u scripts/bench_tpch.py --sf 10 --queries q01,q03,q04,q12,q17,q02 --rounds 2 --no-check --stage-times --json $O/tpch_stages.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
echo done
