# round 5 session: the finest unpooling's two-wave kernel held to two waves per SIMD
# (MSW_UNPOOL_EU2; the eu1 library variant keeps one) -- parity, A/B, traced step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s28; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "f64 or unpool or coop" > $O/tests.log 2>&1 || exit 3
bash tools/ab.sh "" "MSW_LIB_VARIANT=eu1" "" "MSW_LIB_VARIANT=eu1" "" -- --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 || exit 4
cp gpurun_out/ab.log $O/ab.log
timeout -k 10 200 rocprofv3 --kernel-trace -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $O/prof.json 2> $O/prof.err || exit 5
python3 tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step_breakdown.txt 2>&1
rm -f $O/prof/run_kernel_trace.csv
