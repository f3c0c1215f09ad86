#!/bin/bash
# Round 4 (v): kernel trace of TPC-H Q03 at SF10 (the join-build change's effect).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_relops.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_relops.log 2>&1 || { tail -40 $O/pytest_relops.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_q03 -o run --output-format csv -- python3 scripts/bench_tpch.py --sf 10 --queries q03,q12,q04 --rounds 3 --no-check --stage-times > $O/kt_q03.log 2>&1 || { tail -5 $O/kt_q03.log; exit 1; }
grep "^{" $O/kt_q03.log
echo done
