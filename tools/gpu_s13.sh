# round-3 session 13: F = 64 variants (pipelined split edge MLP, blob-read two-wave unpooling):
# bit-identity tests, A/B on zenodo4_f64, a kernel trace of the faster setting
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -x -v -s --timeout 120 --timeout-method thread -k "f64_kernel_variants or train or gradients" > $O/tests.log 2>&1 || exit 3
timeout -k 10 300 python tools/train_bench.py > $O/train_bench.json 2> $O/train_bench.err || exit 8
F="-- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3"
bash tools/ab.sh "MSW_COOP2_DIRECT=0" "" "MSW_MLP_PIPE=1" "MSW_COOP2_DIRECT=0" "" "MSW_MLP_PIPE=1" $F > $O/ab_f64.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_f64 -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 2 > $O/prof_f64.log 2>&1 || exit 5
MSW_MLP_PIPE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_f64_pipe -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 2 > $O/prof_f64_pipe.log 2>&1 || exit 6
echo ok > $O/done
