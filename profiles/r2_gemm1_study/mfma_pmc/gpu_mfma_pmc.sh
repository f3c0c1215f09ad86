# MFMA busy counters of the FF layer-1 GEMM (and shorter-K versions of it, below the 32-bit wrap of the
# summed busy counter) — one counter pass per shape, kernel dispatches only.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/mfma_pmc
for K in 131072 262144 597568; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    -d gpurun_out/mfma_pmc/k$K -o pmc --output-format csv -- python3 scripts/prof_gemm.py 1000 1000 $K 2 6 \
    > gpurun_out/mfma_pmc/k$K.log 2>&1 || exit 1
done
