#!/bin/bash
# BASELINE.json secondary configs on one GPU: LA DSL 64k^2 matmul (config 4 at N=1) and the config-5 dedup
# harness; each step under its own time limit, stop at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/secondary
mkdir -p $O
timeout -k 10 400 python scripts/bench_la_matmul.py --size 65536 --steps 3 > $O/la_64k.json 2> $O/la_64k.err || { tail -20 $O/la_64k.err; exit 1; }
tail -1 $O/la_64k.json
timeout -k 10 400 python scripts/bench_dedup.py > $O/dedup.json 2> $O/dedup.err || { tail -20 $O/dedup.err; exit 1; }
tail -1 $O/dedup.json
