# round-3 session O: the N > 1 bench path on the fused tree, rehearsed with two gloo ranks on
# one GPU (strong-scaling sets 8 and 128, partition / DDP checks as the driver's N = 2 job)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03o; mkdir -p $O
export TMPDIR=/tmp
MSW_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --strong-sets 8,128 > $O/rehearsal2.json 2> $O/rehearsal2.err || exit 7
echo ok > $O/steps.log
