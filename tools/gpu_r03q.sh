# round-3 session Q (final tree): whole GPU suite, smoke, default bench,
# rocprofv3 kernel trace of the bench (the last code change: the opt-in MSW_FUSE_P4 switch)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/bench_prof.json 2> $O/bench_prof.err || exit 6
echo ok >> $O/steps.log
