# round 5 session: encoder state update without per-column selects -- parity, A/B vs the round base
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s21; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 3
bash tools/ab.sh "" "MSW_LIB_VARIANT=r05base" "" "MSW_LIB_VARIANT=r05base" -- --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 5
cp gpurun_out/ab.log $O/ab_zenodo4.log
bash tools/ab.sh "" "MSW_LIB_VARIANT=r05base" "" "MSW_LIB_VARIANT=r05base" -- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 6
cp gpurun_out/ab.log $O/ab_f64.log
