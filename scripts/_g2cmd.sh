set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { tail -30 gpurun_out/pytest_k.log; exit 1; }
tail -2 gpurun_out/pytest_k.log
timeout -k 10 200 python3 scripts/ab_gemm2.py --shapes 1000x14588x64,1000x14588x1000,1000x14588x1024 --cfgs=0,100 --ld-align 8 --rounds 3 > gpurun_out/ab_epi16.log 2>&1 || exit 2
