#!/bin/bash
# A/B of the conv2d job on its own HIP stream vs serial (bench.py --overlap), plus a kernel trace of
# the overlapped step. Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/ov
timeout -k 10 300 python -u -m pytest tests/test_job_streams.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/ov/pytest.log 2>&1 || { tail -30 gpurun_out/ov/pytest.log; exit 1; }
tail -3 gpurun_out/ov/pytest.log
for rep in 1 2; do
  for mode in none after before; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --overlap $mode > gpurun_out/ov/bench_${mode}_$rep.json \
      2> gpurun_out/ov/bench_${mode}_$rep.err || { tail -20 gpurun_out/ov/bench_${mode}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ov/bench_${mode}_$rep.json'));print('$mode',d['value'],d['ms_per_step'])"
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ov/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 4 --warmup 1 --overlap ${PMODE:-after} > gpurun_out/ov/prof.log 2>&1 || { tail -20 gpurun_out/ov/prof.log; exit 1; }
echo done
