#!/bin/bash
# Start-gated conv2d beside the layer-1 GEMM (--overlap beside): tests, interleaved bench A/B, kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/beside
timeout -k 10 300 python -u -m pytest tests/test_job_streams.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/beside/pytest.log 2>&1 || { tail -30 gpurun_out/beside/pytest.log; exit 1; }
tail -2 gpurun_out/beside/pytest.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/beside/none_$r.json 2> /dev/null || exit 1
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --overlap beside > gpurun_out/beside/beside_$r.json 2> gpurun_out/beside/beside_$r.err || { tail -20 gpurun_out/beside/beside_$r.err; exit 1; }
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --overlap beside --reserve-cus 8 > gpurun_out/beside/beside8_$r.json 2> /dev/null || exit 1
done
python3 - <<'PY'
import json
for f in ["none_1","beside_1","beside8_1","none_2","beside_2","beside8_2"]:
    d=json.loads(open(f"gpurun_out/beside/{f}.json").read().strip().splitlines()[-1]); print(f, d["value"], d["ms_per_step"], d["config"]["check"]["ok"])
PY
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/beside/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 10 --overlap beside > gpurun_out/beside/prof.log 2>&1 || { tail -20 gpurun_out/beside/prof.log; exit 1; }
python3 scripts/last_steps.py gpurun_out/beside/prof/run_kernel_trace.csv 12 > gpurun_out/beside/last_steps.txt
cat gpurun_out/beside/last_steps.txt
