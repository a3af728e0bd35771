set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 300 python bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 > gpurun_out/bench_f64.json 2> gpurun_out/bench_f64.err || exit $?
rm -rf gpurun_out/prof_f64
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_f64 -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > gpurun_out/bench_f64_prof.json 2> gpurun_out/bench_f64_prof.err || exit $?
python tools/step_breakdown.py gpurun_out/prof_f64/run_kernel_trace.csv > gpurun_out/step_breakdown_f64.txt
echo done
