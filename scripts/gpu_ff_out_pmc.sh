# MFMA-busy / clock counters of the FF output GEMM (production kernel), one counter pass, dispatches only.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ff_out_pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  -d gpurun_out/ff_out_pmc/pmc -o pmc --output-format csv -- python3 scripts/prof_ff_out.py 10 \
  > gpurun_out/ff_out_pmc/pmc.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/ff_out_pmc/trace -o tr --output-format csv -- \
  python3 scripts/prof_ff_out.py 10 > gpurun_out/ff_out_pmc/trace.log 2>&1 || exit 1
find gpurun_out/ff_out_pmc -name "*.csv" | head
