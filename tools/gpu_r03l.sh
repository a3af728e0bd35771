# round-3 session L: unpooling fused into the fine scale's first edge-MLP + hop launch --
# its bit-identity tests, A/B on zenodo4 and the batch of 8, then the whole GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fused_unpooling or fused_pooling" -x -v --timeout 240 --timeout-method thread > $O/fuse_test.log 2>&1 || { tail -40 $O/fuse_test.log; exit 3; }
bash tools/ab.sh "MSW_UNPOOL_FUSE=0" "MSW_UNPOOL_FUSE=1" "MSW_UNPOOL_FUSE=0" "MSW_UNPOOL_FUSE=1" > $O/ab_z4.txt 2>&1 || exit 4
cp gpurun_out/ab.log $O/ab_z4.log
bash tools/ab.sh "MSW_UNPOOL_FUSE=0" "MSW_UNPOOL_FUSE=1" -- --workload config3 --no-cpu-baseline --steps 5 --warmup 2 > $O/ab_c3.txt 2>&1 || exit 5
cp gpurun_out/ab.log $O/ab_c3.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
cat $O/ab_z4.log $O/ab_c3.log
