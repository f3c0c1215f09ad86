#!/bin/bash
# Round-4 session start: GPU tests, bench, then our GEMM vs hipBLASLt (timing + kernel trace + PMC passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4_vendor
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "[tests]"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  echo "[bench]"; timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
echo "[ab]"; timeout -k 10 300 python -u scripts/ab_vendor_split.py --rounds 5 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
for who in ours blas; do
  for shape in 8k ff; do
    echo "[trace $who $shape]"
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_${who}_${shape} -o run --output-format csv -- python3 scripts/prof_vendor.py $who $shape 5 > $O/kt_${who}_${shape}.log 2>&1 || { tail -5 $O/kt_${who}_${shape}.log; exit 1; }
  done
done
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for who in ours blas; do
    for shape in 8k ff; do
      echo "[pmc $i $who $shape]"
      timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc${i}_${who}_${shape} -o run -- python3 scripts/prof_vendor.py $who $shape 3 > $O/pmc${i}_${who}_${shape}.log 2>&1 || { tail -5 $O/pmc${i}_${who}_${shape}.log; exit 1; }
    done
  done
done
echo "[done]"
