cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/sqf64; mkdir -p $O; export TMPDIR=/tmp
KRE='k_edge_mlp|k_encode|k_edge_coop4|k_hop_split'
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVES --kernel-include-regex "$KRE" -d $PWD/$O/pmc_sq -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 1 --warmup 1 > $O/pmc_sq.log 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$KRE" -d $PWD/$O/pmc_grbm -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 1 --warmup 1 > $O/pmc_grbm.log 2>&1 || exit 4
python3 tools/pmc_generic.py $O/pmc_sq $O/pmc_grbm > $O/pmc_generic.txt 2>&1
