#!/bin/bash
# Round 4 (z4): kernel trace of TPC-H Q01 at SF10.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4z4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_q01 -o run --output-format csv -- python3 scripts/bench_tpch.py --sf 10 --queries q01 --rounds 1 --no-check > $O/kt_q01.log 2>&1 || { tail -5 $O/kt_q01.log; exit 1; }
grep "^{" $O/kt_q01.log
echo done
