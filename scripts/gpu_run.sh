#!/bin/bash
# The one GPU-box runner (gpurun -- bash scripts/gpu_run.sh TASK [TASK ...]). Every task runs under its own time
# limit; the first failure (test failure, abort, fault, timeout) ends the call, so no GPU step runs after one.
#
# Tasks:
#   tests        pytest -m gpu (K=<-k filter> to narrow), per-test timeout, one process
#   smoke        __graft_entry__.smoke()
#   bench        bench.py --steps 20 --warmup 5 (the driver's arguments; BENCH_ARGS overrides)
#   abbench      interleaved bench.py runs of AB_VARIANTS (';'-separated bench argument sets, default the two
#                GEMM MFMA shapes) for AB_ROUNDS rounds (default 5), driver arguments; one JSON line per run
#   prof         rocprofv3 --kernel-trace --stats of bench.py --steps 10 --warmup 10 + per-step timeline
#   pmc          rocprofv3 --pmc pass(es) of bench.py, PMC="counter list" (one pass per ';'-separated list)
#   tpch         scripts/bench_tpch.py at SF 1,10, all ten queries, pandas-checked, stage times (TPCH_ARGS)
#   tpchprof     rocprofv3 kernel trace of scripts/bench_tpch.py (TPCH_ARGS, default SF 10 Q01,Q06)
#   relops       scripts/bench_relops.py (RELOPS_ARGS)
#   relopsprof   rocprofv3 kernel trace of scripts/bench_relops.py (RELOPS_ARGS)
#   secondary    BASELINE.json secondary configs: LA 64k^2 %*%, config-5 dedup harness
#   rccl         the one-rank RCCL test (force_collectives) under rocprofv3, to show the RCCL kernels
#   py           python -u $PY_ARGS (a repo script; PY_LIMIT seconds, default 300)
#   pyprof       the same under rocprofv3 --kernel-trace --stats (kernel summary copied to py_kernel_stats.csv)
# Output under gpurun_out/$TAG (TAG defaults to "run").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-run}
mkdir -p "$O"

fail() { echo "[gpu_run] $1 failed (rc $2)"; [ -f "$3" ] && tail -${4:-40} "$3"; exit "$2"; }

run_task() {
  case "$1" in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${K:+-k "$K"} \
        > "$O/pytest_gpu.log" 2>&1 || fail tests $? "$O/pytest_gpu.log" 60
      tail -3 "$O/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || fail smoke $? "$O/smoke.log"
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > "$O/bench.log" 2>&1 \
        || fail bench $? "$O/bench.log"
      grep "^{" "$O/bench.log" | tee "$O/bench.json" ;;
    abbench)
      IFS=';' read -ra vars <<< "${AB_VARIANTS:---mfma 16;--mfma 32}"
      for r in $(seq 1 "${AB_ROUNDS:-5}"); do
        for v in "${vars[@]}"; do
          timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $v > "$O/ab.log" 2>&1 || fail "abbench ($v)" $? "$O/ab.log"
          echo "{\"round\": $r, \"args\": \"$v\", \"result\": $(grep '^{' "$O/ab.log")}" | tee -a "$O/abbench.jsonl"
        done
      done ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- \
        python3 "$R/bench.py" --steps 10 --warmup 10 ${PROF_ARGS:-} > "$O/prof.log" 2>&1 || fail prof $? "$O/prof.log"
      f=$(ls "$O"/prof/*/run_kernel_stats.csv "$O"/prof/run_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && cp "$f" "$O/bench_kernel_stats.csv" && head -8 "$O/bench_kernel_stats.csv"
      t=$(ls "$O"/prof/*/run_kernel_trace.csv "$O"/prof/run_kernel_trace.csv 2>/dev/null | head -1)
      [ -n "$t" ] && python scripts/timeline.py "$t" 10 > "$O/timeline.txt" && tail -5 "$O/timeline.txt" ;;
    pmc)
      IFS=';' read -ra passes <<< "${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE}"
      i=0
      for p in "${passes[@]}"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $p -d "$R/$O/pmc$i" -o run --output-format csv -- \
          python3 "$R/${PMC_SCRIPT:-bench.py}" ${PMC_ARGS:---steps 5 --warmup 5 --settle-ms 0} > "$O/pmc$i.log" 2>&1 \
          || fail "pmc pass $i" $? "$O/pmc$i.log"
      done
      echo "pmc passes: $i" ;;
    tpch)
      timeout -k 10 1100 python -u scripts/bench_tpch.py ${TPCH_ARGS:---sf 1,10 --queries q01,q02,q03,q04,q06,q12,q13,q14,q17,q22 --stage-times} \
        --json "$O/tpch.json" > "$O/tpch.log" 2>&1 || fail tpch $? "$O/tpch.log"
      grep '^{"sf"' "$O/tpch.log" | tail -12 ;;
    tpchprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/tpchprof" -o run --output-format csv -- \
        python3 "$R/scripts/bench_tpch.py" ${TPCH_ARGS:---sf 10 --queries q01,q06 --rounds 3} > "$O/tpchprof.log" 2>&1 \
        || fail tpchprof $? "$O/tpchprof.log"
      f=$(ls "$O"/tpchprof/*/run_kernel_stats.csv "$O"/tpchprof/run_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && cp "$f" "$O/tpch_kernel_stats.csv" && head -12 "$O/tpch_kernel_stats.csv" ;;
    relops)
      timeout -k 10 600 python -u scripts/bench_relops.py ${RELOPS_ARGS:---rounds 5} --json "$O/relops.json" \
        > "$O/relops.log" 2>&1 || fail relops $? "$O/relops.log"
      grep "^{" "$O/relops.log" | tail -20 ;;
    relopsprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/relopsprof" -o run --output-format csv -- \
        python3 "$R/scripts/bench_relops.py" ${RELOPS_ARGS:---rounds 3} > "$O/relopsprof.log" 2>&1 \
        || fail relopsprof $? "$O/relopsprof.log"
      f=$(ls "$O"/relopsprof/*/run_kernel_stats.csv "$O"/relopsprof/run_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && cp "$f" "$O/relops_kernel_stats.csv" && head -16 "$O/relops_kernel_stats.csv" ;;
    secondary)
      timeout -k 10 400 python scripts/bench_la_matmul.py --size 65536 --steps 3 > "$O/la_64k.json" 2> "$O/la_64k.err" \
        || fail la_64k $? "$O/la_64k.err"
      tail -1 "$O/la_64k.json"
      timeout -k 10 400 python scripts/bench_dedup.py ${DEDUP_ARGS:-} > "$O/dedup.json" 2> "$O/dedup.err" \
        || fail dedup $? "$O/dedup.err"
      tail -1 "$O/dedup.json" ;;
    rccl)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/rccl" -o run --output-format csv -- \
        python3 -m pytest tests/test_force_collectives.py -m gpu -x -q -p no:cacheprovider > "$O/rccl.log" 2>&1 \
        || fail rccl $? "$O/rccl.log"
      f=$(ls "$O"/rccl/*/run_kernel_stats.csv "$O"/rccl/run_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && cp "$f" "$O/rccl_kernel_stats.csv" && grep -i "nccl\|rccl" "$O/rccl_kernel_stats.csv" | head -10 ;;
    py)
      timeout -k 10 "${PY_LIMIT:-300}" python -u $PY_ARGS > "$O/py.log" 2>&1 || fail py $? "$O/py.log"
      tail -${PY_TAIL:-20} "$O/py.log" ;;
    pyprof)
      timeout -k 10 "${PY_LIMIT:-300}" rocprofv3 --kernel-trace --stats -d "$R/$O/pyprof" -o run --output-format csv -- \
        python3 $PY_ARGS > "$O/pyprof.log" 2>&1 || fail pyprof $? "$O/pyprof.log"
      f=$(ls "$O"/pyprof/*/run_kernel_stats.csv "$O"/pyprof/run_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && cp "$f" "$O/py_kernel_stats.csv" && head -${PY_TAIL:-20} "$O/py_kernel_stats.csv" ;;
    *) echo "[gpu_run] unknown task $1"; exit 2 ;;
  esac
}

for t in "$@"; do
  echo "[gpu_run] $t"
  run_task "$t"
done
echo "[gpu_run] done"
