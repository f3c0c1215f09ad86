#!/bin/bash
# A/B: conv2d job serial vs gated into the FF layer-1 GEMM tail (bench.py --overlap tail), interleaved,
# plus a kernel trace of the tail mode. Every GPU step has its own time limit; stop at the first failure.
# CONFIGS: space-separated name=args pairs (args joined by commas), e.g. "none=--overlap,none tail=--overlap,tail"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/ab_tail
mkdir -p $O
CONFIGS=${CONFIGS:-"none=--overlap,none tail=--overlap,tail"}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_job_streams.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2; do
  for c in $CONFIGS; do
    n=${c%%=*}; a=${c#*=}; a=${a//,/ }
    timeout -k 10 300 python bench.py $a > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || { tail -20 $O/bench_${n}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/bench_${n}_$r.json')); print('$n', d['value'], d['ms_per_step'], d['config']['check']['ok'])"
  done
done
if [ -n "$PROF_ARGS" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" ${PROF_ARGS//,/ } --steps 10 --warmup 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  python scripts/timeline.py $O/prof/run_kernel_trace.csv 16
fi
echo done
