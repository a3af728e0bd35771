# round-3 session 18: bias gradients fused into the weight-gradient GEMM -- training tests and
# training-step time
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s18; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 3
timeout -k 10 400 python tools/train_bench.py > $O/train_bench.json 2> $O/train_bench.err || exit 4
echo ok > $O/done
