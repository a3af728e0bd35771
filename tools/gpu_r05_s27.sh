# round 5 session: the finest unpooling's F = 64 kernel choice (plain / two-wave blob-read /
# two-wave LDS-staged) on the final library, with a traced step per setting
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s27; mkdir -p $O
bash tools/ab.sh "" "MSW_COOP2_DIRECT=0" "MSW_COOP2_DIRECT=2" "MSW_COOP2_F64=0" "MSW_COOP_WAVES=8192" "" -- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 4
cp gpurun_out/ab.log $O/ab_f64_unpool.log
for e in MSW_COOP2_DIRECT=2 MSW_COOP_WAVES=8192; do
  env $e timeout -k 10 200 rocprofv3 --kernel-trace -d $PWD/$O/prof_$e -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $O/prof_$e.json 2> $O/prof_$e.err || exit 5
  python3 tools/step_breakdown.py $O/prof_$e/run_kernel_trace.csv > $O/step_breakdown_$e.txt 2>&1
  rm -f $O/prof_$e/run_kernel_trace.csv
done
