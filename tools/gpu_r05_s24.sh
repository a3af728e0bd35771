# round 5 session: split edge MLP gathers its first chunk during the weight staging -- parity, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s24; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 3
bash tools/ab.sh "" "MSW_LIB_VARIANT=r05base" "" "MSW_LIB_VARIANT=r05base" -- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 4
cp gpurun_out/ab.log $O/ab_f64.log
