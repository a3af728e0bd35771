# round 5 session: parity suite + F = 64 and zenodo4 lines with the split edge MLP stagger on by default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s23; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 3
bash tools/ab.sh "" "MSW_MLP_STAGGER=0" "" "MSW_MLP_STAGGER=0" -- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 4
cp gpurun_out/ab.log $O/ab_f64.log
