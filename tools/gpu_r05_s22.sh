# round 5 session: stagger of the split edge MLP's waves (F = 64)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s22; mkdir -p $O
bash tools/ab.sh "" "MSW_MLP_STAGGER=1" "MSW_MLP_STAGGER=2" "MSW_MLP_STAGGER=4" "MSW_MLP_STAGGER=8" "" "MSW_MLP_STAGGER=2" "MSW_MLP_STAGGER=4" -- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 4
cp gpurun_out/ab.log $O/ab_f64_stagger.log
