# round 5 session: re-check the F = 64 switches' defaults on the final library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s25; mkdir -p $O
bash tools/ab.sh "" "MSW_HOP_ROWS=2" "MSW_HOP_SPLIT=0" "MSW_ENC_COOP=0" "MSW_SPLIT_EDGE_MLP=0" "MSW_POOL_WIDE=0" "MSW_COOP_WAVES=0" "" -- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 4
cp gpurun_out/ab.log $O/ab_f64_switches.log
