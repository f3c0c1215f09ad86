#!/bin/bash
# Round 4 (m): full GPU suite (incl. two-rank TPC-H on one GPU), headline bench, smoke.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4m
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu suite]"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[smoke]"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[bench]"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log
echo done
