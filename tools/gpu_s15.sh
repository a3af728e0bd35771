# round-3 session 15: training path with HIP encoders / decoder / pooling -- gradient tests,
# training-step timing, kernel stats of the HIP training step
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s15; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "train or gradients or f64_kernel_variants or grid_stride" > $O/tests.log 2>&1 || exit 3
timeout -k 10 300 python tools/train_bench.py > $O/train_bench.json 2> $O/train_bench.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_train -o run --output-format csv -- python3 tools/train_bench.py --only hip --steps 3 --warmup 1 > $O/prof_train.log 2>&1 || exit 5
echo ok > $O/done
