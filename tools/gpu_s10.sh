set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -v -s --timeout 500 --timeout-method thread -k config3 > $O/config3_tests.log 2>&1
echo "config3 rc=$?" >> $O/steps.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_f64 -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $O/bench_f64_prof.json 2> $O/prof.err || exit 5
echo ok >> $O/steps.log
