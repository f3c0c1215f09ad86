#!/bin/bash
# w4a diagnostics: interleaved A/B of the production 8-phase kernel, the w4a schedule and its ablations
# (no global loads / no LDS writes / no barriers / no fragment reads), then one PMC pass per kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/w4a_pmc
timeout -k 10 300 python -u scripts/ab_w4a.py --cfgs ${CFGS:-2,30,33,34,35,36} --rounds 4 --shapes ff,8192 > gpurun_out/ab_w4a_diag.log 2>&1
rc=$?; tail -4 gpurun_out/ab_w4a_diag.log; [ $rc -ne 0 ] && exit $rc
for c in 2 30; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    -d gpurun_out/w4a_pmc/c$c -o pmc --output-format csv -- python3 scripts/prof_gemm.py 8192 8192 8192 $c 4 \
    > gpurun_out/w4a_pmc/c$c.log 2>&1 || { tail -5 gpurun_out/w4a_pmc/c$c.log; exit 1; }
done
echo pmc done
