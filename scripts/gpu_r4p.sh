#!/bin/bash
# Round 4 (p): the two-rank TPC-H GPU test alone (per-rank tracebacks), then the rest of the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4p
mkdir -p $O
export TMPDIR=/tmp
echo "[two-rank test]"
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1 || { grep -v "^E  *$" $O/pytest_dist.log | grep -A40 "rank failures" | head -80; exit 1; }
tail -2 $O/pytest_dist.log
echo "[gpu suite]"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_distributed_gpu.py::test_tpch_two_ranks_on_one_gpu_vs_pandas > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[smoke]"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[bench]"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log
echo done
