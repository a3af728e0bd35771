set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s9; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v -s --timeout 200 --timeout-method thread > $O/gpu_train.log 2>&1 || exit 4
timeout -k 10 600 python tools/train_bench.py > $O/train_bench.json 2> $O/train_bench.err || exit 5
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_hip -o run --output-format csv -- python3 tools/train_bench.py --only hip --steps 3 --warmup 1 > $O/train_hip.json 2> $O/prof_hip.err || exit 6
echo ok
