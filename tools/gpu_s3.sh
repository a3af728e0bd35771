set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v -s --timeout 300 --timeout-method thread > $O/gpu_train.log 2>&1
echo "rc=$?" >> $O/gpu_train.log
