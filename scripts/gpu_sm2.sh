#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/sm
timeout -k 10 300 python -u -m pytest tests/test_softmax_gemm.py tests/test_headline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sm/pytest.log 2>&1 || { tail -30 gpurun_out/sm/pytest.log; exit 1; }
tail -2 gpurun_out/sm/pytest.log
timeout -k 10 180 python scripts/prof_softmax_stamps.py > gpurun_out/sm/stamps.json 2> gpurun_out/sm/stamps.err || { tail -20 gpurun_out/sm/stamps.err; exit 1; }
timeout -k 10 180 python scripts/ab_ff_tail.py > gpurun_out/sm/ab_ff_tail.log 2>&1 || { tail -20 gpurun_out/sm/ab_ff_tail.log; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/sm/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 10 --single-job > gpurun_out/sm/prof.log 2>&1 || { tail -20 gpurun_out/sm/prof.log; exit 1; }
python3 scripts/last_steps.py gpurun_out/sm/prof/run_kernel_trace.csv 12 > gpurun_out/sm/last_steps.txt
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/sm/two_$r.json 2> /dev/null || exit 1
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --single-job > gpurun_out/sm/one_$r.json 2> /dev/null || exit 1
done
python3 - <<'PY'
import json
for f in ["two_1","one_1","two_2","one_2"]:
    d=json.loads(open(f"gpurun_out/sm/{f}.json").read().strip().splitlines()[-1]); print(f, d["value"], d["ms_per_step"], d["config"]["check"]["ff_max_rel_err"])
PY
python3 -c "import json;d=json.load(open('gpurun_out/sm/stamps.json'.replace('.json','.json')))" 2>/dev/null; cat gpurun_out/sm/ab_ff_tail.log gpurun_out/sm/last_steps.txt
