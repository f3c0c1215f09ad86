#!/bin/bash
# Round 4 (ov): headline A/B on one box — conv2d job serial (default) vs on its own stream after / before the FF jobs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4ov
mkdir -p $O
for mode in none after before none after; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --overlap $mode > $O/bench_$mode.log 2>&1 || { tail -20 $O/bench_$mode.log; exit 1; }
  echo "$mode $(grep '^{' $O/bench_$mode.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
echo done
