# round-3 session I: pooling fused into the coarse scales' first edge-MLP + hop launch --
# its bit-identity test first, then the whole GPU suite, then A/B (MSW_POOL_FUSE=0 / 1)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k fused_pooling -x -v --timeout 240 --timeout-method thread > $O/fuse_test.log 2>&1 || { tail -30 $O/fuse_test.log; exit 3; }
AB_KEEP=1 bash tools/ab.sh "MSW_POOL_FUSE=0" "MSW_POOL_FUSE=1" "MSW_POOL_FUSE=0" "MSW_POOL_FUSE=1" > $O/ab_z4.txt 2>&1 || exit 4
AB_KEEP=1 bash tools/ab.sh "MSW_POOL_FUSE=0" "MSW_POOL_FUSE=1" -- --workload config3 --no-cpu-baseline --steps 5 --warmup 2 > $O/ab_c3.txt 2>&1 || exit 5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
cat gpurun_out/ab.log
