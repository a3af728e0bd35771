# round-3 session B: PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs), the config-3 parity test,
# extra workloads
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03b; mkdir -p $O
export TMPDIR=/tmp
KRE='k_hop|k_edge_hop|k_pool|k_encode'
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $PWD/$O/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1 || exit 4
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $PWD/$O/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc_write.log 2>&1 || exit 5
python3 tools/pmc_summary.py $O/pmc_summary.json $O/pmc_fetch $O/pmc_write > $O/pmc_summary.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -v -s --timeout 500 --timeout-method thread -k config3 > $O/config3_tests.log 2>&1
echo "config3 rc=$?" >> $O/steps.log
timeout -k 10 300 python bench.py --workload hbm1m --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_hbm1m.json 2> $O/bench_hbm1m.err || exit 6
timeout -k 10 300 python bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 > $O/bench_f64.json 2> $O/bench_f64.err || exit 7
echo ok >> $O/steps.log
