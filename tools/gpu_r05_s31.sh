# round 5 session: start stagger of the F = 64 cooperative encoder's co-resident workgroups
# (MSW_ENC_STAGGER = n: workgroup b sleeps ((b >> 8) & 3) x n x 2 k cycles after its first loads)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s31; mkdir -p $O
bash tools/ab.sh "" "MSW_ENC_STAGGER=1" "MSW_ENC_STAGGER=2" "MSW_ENC_STAGGER=4" "" "MSW_ENC_STAGGER=2" "MSW_ENC_STAGGER=1" -- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 4
cp gpurun_out/ab.log $O/ab_enc_stagger.log
