#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py for each ARGSETS entry (args joined by commas), per-step timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/prof_bench
mkdir -p $O
i=0
for a in ${ARGSETS:-"--overlap,none"}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/p$i" -o run --output-format csv -- python3 "$R/bench.py" ${a//,/ } --steps 10 --warmup 10 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  echo "== $a"; python scripts/timeline.py $O/p$i/run_kernel_trace.csv 10
done
