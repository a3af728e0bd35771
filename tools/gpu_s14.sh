# round-3 session 14: grid-stride edge hop with the next tile's record prefetched -- parity
# (forced loop == one tile per wave) and A/B on the ~1M-node mesh against the no-prefetch build
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s14; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "grid_stride_edge_hops" > $O/tests.log 2>&1 || exit 3
H="-- --workload hbm1m --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1"
bash tools/ab.sh "MSW_LIB_VARIANT=ehnopf" "" "MSW_LIB_VARIANT=ehnopf" "" $H > $O/ab_hbm1m.log 2>&1 || exit 4
bash tools/ab.sh "MSW_LIB_VARIANT=ehnopf" "" -- --no-cpu-baseline --steps 10 --warmup 3 > $O/ab_zenodo4.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_hbm1m -o run --output-format csv -- python3 bench.py --workload hbm1m --no-cpu-baseline --no-roofline-large --steps 2 --warmup 1 > $O/prof_hbm1m.log 2>&1 || exit 6
echo ok > $O/done
