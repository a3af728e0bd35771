# round 5 session: the cooperative-kernel size rule (MSW_COOP_WAVES) re-checked on the headline
# workload with the final library (the finest unpooling, 652 tiles, is just above the default 1024)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s30; mkdir -p $O
bash tools/ab.sh "" "MSW_COOP_WAVES=1536" "MSW_COOP_WAVES=2048" "MSW_COOP_WAVES=4096" "MSW_COOP_WAVES=768" "" "MSW_COOP_WAVES=1536" -- --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 4
cp gpurun_out/ab.log $O/ab_coop_waves.log
MSW_COOP_WAVES=1536 timeout -k 10 200 rocprofv3 --kernel-trace -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $O/prof.json 2> $O/prof.err || exit 5
python3 tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step_breakdown_cw1536.txt 2>&1
rm -f $O/prof/run_kernel_trace.csv
