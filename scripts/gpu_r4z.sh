#!/bin/bash
# Round 4 (z): Q12 fused group-by fallback diagnosis.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 300 python -u scripts/debug_q12_groupby.py > $O/debug.log 2>&1 || { tail -30 $O/debug.log; exit 1; }
grep -v "^$" $O/debug.log | tail -30
