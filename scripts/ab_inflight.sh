#!/bin/bash
# FF steps in flight (bench.py --inflight) A/B, with the conv2d job overlapped; kernel trace of inflight=2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/inf
timeout -k 10 300 python -u -m pytest tests/test_job_streams.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/inf/pytest.log 2>&1 || { tail -30 gpurun_out/inf/pytest.log; exit 1; }
for rep in 1 2; do
  for n in 1 2 3; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 3 --inflight $n > gpurun_out/inf/bench_i${n}_$rep.json \
      2> gpurun_out/inf/bench_i${n}_$rep.err || { tail -20 gpurun_out/inf/bench_i${n}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/inf/bench_i${n}_$rep.json'));print('inflight $n',d['value'],d['ms_per_step'],d['config']['softmax_rows_sum_to_1'])"
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/inf/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 6 --warmup 2 --inflight 2 > gpurun_out/inf/prof.log 2>&1 || { tail -20 gpurun_out/inf/prof.log; exit 1; }
echo done
