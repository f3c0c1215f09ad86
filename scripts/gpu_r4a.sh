#!/bin/bash
# Round 4: device relational operators (tests + micro-bench), then the GEMM vendor comparison.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
echo "[relops tests]"
timeout -k 10 300 python -u -m pytest tests/test_relops.py tests/test_strings.py tests/test_hashagg.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_relops.log 2>&1 || { tail -40 $O/pytest_relops.log; exit 1; }
tail -3 $O/pytest_relops.log
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/bench_relops.json > $O/bench_relops.log 2>&1 || { tail -30 $O/bench_relops.log; exit 1; }
cat $O/bench_relops.log
echo "[tpch sf1]"
timeout -k 10 600 python -u scripts/bench_tpch.py --sf ${TPCH_SF:-1} --rounds 3 --json $O/tpch.json > $O/tpch.log 2>&1 || { tail -30 $O/tpch.log; exit 1; }
cat $O/tpch.log
echo "[engine gpu tests]"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
SKIP_TESTS=1 bash scripts/gpu_vendor_pmc.sh
