# Interleaved bench A/B: the reference's two-job inference_unit (default) vs --single-job (fused softmax GEMM).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/single_job
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/single_job/two_$r.json 2> gpurun_out/single_job/two_$r.err || exit 1
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --single-job > gpurun_out/single_job/one_$r.json 2> gpurun_out/single_job/one_$r.err || exit 1
done
