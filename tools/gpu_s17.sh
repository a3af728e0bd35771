# round-3 session 17: training gradients of the HIP path and of torch's fp32 path against the
# torch path in float64 (exact-arithmetic yardstick), 1- and 4-step training rollouts
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s17; mkdir -p $O
: > $O/fp64.jsonl
for r in 1 4; do
  timeout -k 10 400 python tools/train_bench.py --rollout-steps $r --fp64-ref --steps 1 --warmup 0 >> $O/fp64.jsonl 2> $O/fp64.err || exit 3
done
echo ok > $O/done
