# round-3 session M: fused unpooling at F = 64 (k_edge_coop4 FUSE=2) -- bit-identity tests,
# A/B on zenodo4_f64, then the whole GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fused_unpooling" -x -v --timeout 240 --timeout-method thread > $O/fuse_test.log 2>&1 || { tail -40 $O/fuse_test.log; exit 3; }
bash tools/ab.sh "MSW_UNPOOL_FUSE=0" "MSW_UNPOOL_FUSE=1" "MSW_UNPOOL_FUSE=0" "MSW_UNPOOL_FUSE=1" -- --workload zenodo4_f64 --no-cpu-baseline --steps 10 --warmup 3 > $O/ab_f64.txt 2>&1 || exit 4
cp gpurun_out/ab.log $O/ab_f64.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
cat $O/ab_f64.log
