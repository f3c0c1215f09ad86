#!/bin/bash
# Round 4 (b): full GPU suite, then rocprof kernel traces of the relational micro-bench and TPC-H SF1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests]"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[relops trace]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/relops_prof -o run --output-format csv -- python3 scripts/bench_relops.py --rounds 2 > $O/relops_prof.log 2>&1 || { tail -20 $O/relops_prof.log; exit 1; }
echo "[tpch trace]"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/tpch_prof -o run --output-format csv -- python3 scripts/bench_tpch.py --sf 1 --rounds 1 --no-check > $O/tpch_prof.log 2>&1 || { tail -20 $O/tpch_prof.log; exit 1; }
cat $O/tpch_prof.log | tail -8
echo "[bench]"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
SKIP_TESTS=1 bash scripts/gpu_vendor_pmc.sh
