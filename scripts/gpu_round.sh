#!/bin/bash
# One GPU session: kernel/engine GPU tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
echo "[gpu_round] tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
echo "[gpu_round] smoke" && timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo "[gpu_round] bench" && timeout -k 10 600 python bench.py --steps ${STEPS:-50} --warmup ${WARMUP:-10} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ "${PROFILE:-1}" = "1" ]; then
  echo "[gpu_round] rocprofv3"
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 10 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
