#!/bin/bash
# Round 4 (f): relops tests, kernel traces + PMC of the aggregation kernels at 10k / 10M distinct keys.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu tests: relops]"
timeout -k 10 300 python -u -m pytest tests/test_relops.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for d in 8 10000 10000000; do
  echo "[trace $d]"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$d -o run --output-format csv -- python3 scripts/prof_relops_case.py $d 3 > $O/kt_$d.log 2>&1 || { tail -5 $O/kt_$d.log; exit 1; }
done
for d in 10000 10000000; do
  echo "[pmc $d]"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1_$d -o run -- python3 scripts/prof_relops_case.py $d 2 > $O/pmc1_$d.log 2>&1 || { tail -5 $O/pmc1_$d.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2_$d -o run -- python3 scripts/prof_relops_case.py $d 2 > $O/pmc2_$d.log 2>&1 || { tail -5 $O/pmc2_$d.log; exit 1; }
done
echo "[relops bench]"
timeout -k 10 300 python -u scripts/bench_relops.py --rounds 5 --json $O/relops.json > $O/relops.log 2>&1 || { tail -20 $O/relops.log; exit 1; }
grep "^{" $O/relops.log
echo "[tpch sf1 + host profile]"
timeout -k 10 400 python -u scripts/bench_tpch.py --sf 1 --rounds 3 --json $O/tpch.json --host-profile $O/hostprof > $O/tpch.log 2>&1 || { tail -20 $O/tpch.log; exit 1; }
grep "^{" $O/tpch.log
echo "[dedup bench]"
timeout -k 10 300 python -u scripts/bench_dedup.py > $O/dedup.json 2> $O/dedup.err || { tail -20 $O/dedup.err; exit 1; }
cat $O/dedup.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dedup_prof -o run --output-format csv -- python3 scripts/bench_dedup.py --steps 3 --warmup 1 > $O/dedup_prof.log 2>&1 || { tail -20 $O/dedup_prof.log; exit 1; }
echo done
