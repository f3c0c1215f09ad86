#!/bin/bash
# Round 4 (k): relops tests + bench, headline bench (driver args) and its kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4k
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops]"
timeout -k 10 300 python -u -m pytest tests/test_relops.py tests/test_tpch.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
echo "[bench]"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "[bench trace]"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bench_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 10 > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
echo done
