set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/bench_services.py --device cuda:0 > gpurun_out/bench_services.log 2>&1 || { tail -20 gpurun_out/bench_services.log; exit 1; }
grep primitive gpurun_out/bench_services.log
