# round-3 final session E: PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs), the other
# workloads' bench lines, the F = 64 kernel trace, the training step
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03e; mkdir -p $O
export TMPDIR=/tmp
KRE='k_hop|k_edge_hop|k_pool|k_encode'
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $PWD/$O/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1 || exit 4
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $PWD/$O/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc_write.log 2>&1 || exit 5
python3 tools/pmc_summary.py $O/pmc_summary.json $O/pmc_fetch $O/pmc_write > $O/pmc_summary.log 2>&1
timeout -k 10 300 python bench.py --workload hbm1m --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_hbm1m.json 2> $O/bench_hbm1m.err || exit 6
timeout -k 10 300 python bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 > $O/bench_f64.json 2> $O/bench_f64.err || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_f64 -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 2 > $O/prof_f64.log 2>&1 || exit 8
timeout -k 10 300 python bench.py --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 5 --warmup 2 > $O/bench_refloop.json 2> $O/bench_refloop.err || exit 9
bash tools/ab.sh "" "MSW_ENC_COOP_P=2" "" "MSW_ENC_COOP_P=2" -- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 > $O/ab_enc_p2.log 2>&1 || exit 11
timeout -k 10 400 python tools/train_bench.py > $O/train_bench.json 2> $O/train_bench.err || exit 10
echo ok >> $O/steps.log
