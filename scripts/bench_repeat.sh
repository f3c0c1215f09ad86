#!/bin/bash
# bench.py A/B with a long warmup (clock ramp excluded): serial vs conv2d job on its own stream.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/rep
i=0
for args in "--overlap none" "--overlap before" "--overlap none" "--overlap before" "--overlap none" "--overlap before" "--overlap after --steps 100"  "--overlap none --steps 100"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 $args > gpurun_out/rep/c$i.json 2> gpurun_out/rep/c$i.err || { tail -20 gpurun_out/rep/c$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/rep/c$i.json'));print('$i [$args]',d['value'],d['ms_per_step'])"
done
