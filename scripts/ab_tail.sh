#!/bin/bash
# A/B: conv2d job serial vs gated into the FF layer-1 GEMM tail (bench.py --overlap tail), interleaved,
# plus a kernel trace of the tail mode. Every GPU step has its own time limit; stop at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/ab_tail
timeout -k 10 300 python -u -m pytest tests/test_job_streams.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ab_tail/pytest.log 2>&1
rc=$?; tail -6 gpurun_out/ab_tail/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for m in none tail ${EXTRA_MODES}; do
    timeout -k 10 300 python bench.py --overlap $m ${BENCH_ARGS} > gpurun_out/ab_tail/bench_${m}_$r.json 2> gpurun_out/ab_tail/bench_${m}_$r.err || { tail -20 gpurun_out/ab_tail/bench_${m}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_tail/bench_${m}_$r.json')); print('$m', d['value'], d['ms_per_step'], d['config']['check']['ok'])"
  done
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ab_tail/prof" -o run --output-format csv -- python3 "$R/bench.py" --overlap tail --steps 10 --warmup 10 > gpurun_out/ab_tail/prof.log 2>&1 || { tail -20 gpurun_out/ab_tail/prof.log; exit 1; }
echo done
