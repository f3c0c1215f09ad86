#!/bin/bash
# Direct split-K slab epilogue + in-kernel operand prefetch: kernel tests, isolated A/B, interleaved bench A/B,
# kernel trace of the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/pf
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_variants_gpu.py tests/test_headline_gpu.py tests/test_softmax_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pf/pytest.log 2>&1 || { tail -30 gpurun_out/pf/pytest.log; exit 1; }
tail -2 gpurun_out/pf/pytest.log
timeout -k 10 300 python scripts/ab_gemm1_epi.py > gpurun_out/pf/ab_gemm1_epi.log 2>&1 || { tail -20 gpurun_out/pf/ab_gemm1_epi.log; exit 1; }
cat gpurun_out/pf/ab_gemm1_epi.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/pf/pf_$r.json 2> /dev/null || exit 1
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-operand-prefetch > gpurun_out/pf/nopf_$r.json 2> /dev/null || exit 1
done
python3 - <<'PY'
import json
for f in ["pf_1","nopf_1","pf_2","nopf_2"]:
    d=json.loads(open(f"gpurun_out/pf/{f}.json").read().strip().splitlines()[-1]); print(f, d["value"], d["ms_per_step"], d["config"]["check"]["ok"])
PY
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pf/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 10 > gpurun_out/pf/prof.log 2>&1 || { tail -20 gpurun_out/pf/prof.log; exit 1; }
python3 scripts/last_steps.py gpurun_out/pf/prof/run_kernel_trace.csv 12 > gpurun_out/pf/last_steps.txt
cat gpurun_out/pf/last_steps.txt
