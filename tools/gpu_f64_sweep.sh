#!/bin/bash
# F = 64 (verdict r3 item 5): kernel trace of zenodo4_f64 on the current library (step
# breakdown), then a same-box A/B of plan switches that move its launches around (each run
# has its own time limit; a failure stops the script).   bash tools/gpu_f64_sweep.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-f64}
mkdir -p $OUT
export TMPDIR=/tmp
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 3
python3 tools/step_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/step_breakdown_f64.txt
export AB_KEEP=1
: > gpurun_out/ab.log
A="--no-cpu-baseline --no-roofline-large --steps 10 --warmup 3"
bash tools/ab.sh "" "MSW_EPI_SPLIT_TILES=1024" "MSW_XCD_MAX=4" "MSW_COOP_WAVES=16384" "" "MSW_EPI_SPLIT_TILES=1024" "MSW_XCD_MAX=4" "MSW_COOP_WAVES=16384" -- --workload zenodo4_f64 $A || exit 4
bash tools/ab.sh "" "MSW_EPI_SPLIT_TILES=1024" "" "MSW_EPI_SPLIT_TILES=1024" -- $A || exit 5
cp gpurun_out/ab.log $OUT/ab_f64_sweep.txt
echo done >> $OUT/ab_f64_sweep.txt
