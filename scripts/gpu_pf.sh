#!/bin/bash
# Tail prefetch session: cold-operand A/B, the headline FF test (prefetch happened, bit-identical without), and an
# interleaved bench A/B with / without the prefetch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_cold_operands.py > gpurun_out/ab_cold.log 2>&1 || { cat gpurun_out/ab_cold.log; exit 1; }
cat gpurun_out/ab_cold.log
timeout -k 10 400 python -u -m pytest tests/test_headline_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/headline.log 2>&1
rc=$?; tail -3 gpurun_out/headline.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/headline.log; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_pf_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-tail-prefetch > gpurun_out/bench_nopf_$i.json 2>/dev/null || exit 1
  python -c "import json;a=json.load(open('gpurun_out/bench_pf_$i.json'));b=json.load(open('gpurun_out/bench_nopf_$i.json'));print('pf',a['value'],a['ms_per_step'],'nopf',b['value'],b['ms_per_step'])"
done
