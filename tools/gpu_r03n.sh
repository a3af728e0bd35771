# round-3 session N (after the (un)pooling fusions): whole GPU suite, smoke, default bench,
# rocprofv3 kernel trace of the bench, F = 64 / batch-of-8 / config-5 / reference-loop lines
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?" >> $O/steps.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/bench_prof.json 2> $O/bench_prof.err || exit 6
timeout -k 10 300 python bench.py --workload zenodo4_f64 --no-cpu-baseline > $O/bench_f64.json 2> $O/bench_f64.err || exit 7
timeout -k 10 300 python bench.py --workload config3 --no-cpu-baseline > $O/bench_config3.json 2> $O/bench_config3.err || exit 8
timeout -k 10 300 python bench.py --caller reference-loop --no-cpu-baseline > $O/bench_refloop.json 2> $O/bench_refloop.err || exit 9
timeout -k 10 300 python bench.py --workload hbm1m --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_hbm1m.json 2> $O/bench_hbm1m.err || exit 10
echo ok >> $O/steps.log
