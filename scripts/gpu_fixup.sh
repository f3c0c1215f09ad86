set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_variants_gpu.py -k "fixup or ksteal" > gpurun_out/fx_test.log 2>&1 && \
timeout -k 10 300 python -u scripts/ab_fixup.py --rounds 7 > gpurun_out/fx_ab.log 2>&1
