#!/bin/bash
# Round 4 (final 3): validation after the single-part concat fixes — full GPU suite, smoke, headline bench, TPC-H all ten at SF1 / SF10 (checked,
# stage times), relops bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4final3
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu suite]"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[smoke]"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[bench]"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log
echo "[tpch]"
timeout -k 10 900 python -u scripts/bench_tpch.py --sf 1,10 --queries q01,q02,q03,q04,q06,q12,q13,q14,q17,q22 --stage-times --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{\"sf\"" $O/tpch.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
echo done
