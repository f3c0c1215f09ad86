#!/bin/bash
# conv2d job-stream priority A/B (bench.py --job-priority), then the full GPU test suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/pr
for rep in 1 2; do
  for pr in 0 -1; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 3 --job-priority=$pr > gpurun_out/pr/bench_p${pr}_$rep.json \
      2> gpurun_out/pr/bench_p${pr}_$rep.err || { tail -20 gpurun_out/pr/bench_p${pr}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/pr/bench_p${pr}_$rep.json'));print('prio $pr',d['value'],d['ms_per_step'])"
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pr/pytest_gpu.log 2>&1 \
  || { tail -30 gpurun_out/pr/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pr/pytest_gpu.log
