set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "captured_forward or stepped or dropin" > $O/gpu_tests.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 10 --warmup 2 > $O/bench_refloop.json 2> $O/bench_refloop.err || exit 5
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 2 --warmup 1 > $O/bench_refloop_prof.json 2> $O/prof.err || exit 6
echo ok
