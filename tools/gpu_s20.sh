# round-3 session 20: training tests (batched step), F = 64 encoder on two waves per tile (parity, A/B)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s20; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -x -v -s --timeout 200 --timeout-method thread -k "train or gradients or coop_encoder" > $O/tests.log 2>&1 || exit 3
F="-- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3"
bash tools/ab.sh "" "MSW_ENC_COOP_P=2" "" "MSW_ENC_COOP_P=2" $F > $O/ab_f64.log 2>&1 || exit 4
echo ok > $O/done
