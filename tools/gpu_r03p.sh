# round-3 session P: F = 64 after the fused pooling -- kernel trace of the zenodo4_f64 bench,
# and A/B of the fused scale-1 launch on four waves per tile with a blob-read MLP region
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --steps 5 --warmup 1 > $O/bench_prof.json 2> $O/bench_prof.err || exit 6
bash tools/ab.sh "MSW_FUSE_P4=0" "MSW_FUSE_P4=1" "MSW_FUSE_P4=0" "MSW_FUSE_P4=1" -- --workload zenodo4_f64 --no-cpu-baseline --steps 10 --warmup 3 > $O/ab.txt 2>&1 || exit 4
cp gpurun_out/ab.log $O/ab.log
MSW_FUSE_P4=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fused_pooling" -x -v --timeout 240 --timeout-method thread > $O/fuse_test_p4.log 2>&1
echo "p4 tests rc=$?" >> $O/steps.log
cat $O/ab.log
