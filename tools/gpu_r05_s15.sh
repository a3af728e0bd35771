# round 5 session: stagger of the grid-stride fused edge MLP + hop's waves (config 5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s15; mkdir -p $O
bash tools/ab.sh "" "MSW_EH_STAGGER=1" "MSW_EH_STAGGER=2" "MSW_EH_STAGGER=4" "" "MSW_EH_STAGGER=1" "MSW_EH_STAGGER=2" "MSW_EH_STAGGER=4" -- --workload hbm1m --no-cpu-baseline --steps 5 --warmup 2 || exit 4
cp gpurun_out/ab.log $O/ab_hbm1m_stagger.log
