#!/bin/bash
# Round 4 (y): host profiles (cProfile) of TPC-H Q01 / Q12 / Q17 at SF10.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_tpch.py --sf 10 --queries q01,q12,q17 --rounds 2 --no-check --host-profile $O/hostprof > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo done
