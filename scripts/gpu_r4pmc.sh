#!/bin/bash
# Round 4 (pmc): counters of the PART group-by kernels at 10 K keys / 16 M rows (one pass, SQ + GRBM only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r4pmc
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --stats -d $O/pmc -o run --output-format csv -- python3 scripts/prof_relops_case.py 10000 2 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
ls $O/pmc
echo done
