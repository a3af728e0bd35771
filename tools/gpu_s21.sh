# round-3 session 21: training tests + training-step time with cached descriptors (two runs)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s21; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 3
timeout -k 10 400 python tools/train_bench.py > $O/train_bench.json 2> $O/train_bench.err || exit 4
timeout -k 10 400 python tools/train_bench.py --only hip --steps 10 --warmup 3 > $O/train_hip.json 2>> $O/train_bench.err || exit 5
echo ok > $O/done
