set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 scripts/rehearse_meta_group.py > gpurun_out/meta_group.log 2>&1; rc=$?
grep "rank" gpurun_out/meta_group.log | tail -4; tail -5 gpurun_out/meta_group.log; exit $rc
