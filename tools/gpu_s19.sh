# round-3 session 19: training tests + kernel time of the HIP training step (bias fusion)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s19; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_train -o run --output-format csv -- python3 tools/train_bench.py --only hip --steps 3 --warmup 1 > $O/prof_train.log 2>&1 || exit 5
echo ok > $O/done
