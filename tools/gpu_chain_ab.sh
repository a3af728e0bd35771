#!/bin/bash
# Same-box A/B of the persistent middle-hop chains (MSW_HOP_CHAIN = 0 / 1 / 2) on the
# Zenodo-size workloads, interleaved twice, then a rocprofv3 kernel trace of the default
# workload with the best setting (step breakdown).   bash tools/gpu_chain_ab.sh OUTDIR [BEST]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-chain}
BEST=${2:-2}
mkdir -p $OUT
export AB_KEEP=1
: > gpurun_out/ab.log
A="--no-cpu-baseline --no-roofline-large --steps 20 --warmup 3"
bash tools/ab.sh "" "MSW_HOP_CHAIN=1" "MSW_HOP_CHAIN=2" "" "MSW_HOP_CHAIN=1" "MSW_HOP_CHAIN=2" -- $A || exit $?
bash tools/ab.sh "" "MSW_HOP_CHAIN=$BEST" -- --workload zenodo3 $A || exit $?
bash tools/ab.sh "" "MSW_HOP_CHAIN=$BEST" -- --workload zenodo4 --batch 8 $A || exit $?
bash tools/ab.sh "" "MSW_HOP_CHAIN=$BEST" -- --workload dk15 --T 200 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 || exit $?
bash tools/ab.sh "" "MSW_HOP_CHAIN=$BEST" -- --workload zenodo4_f64 $A || exit $?
bash tools/ab.sh "" "MSW_HOP_CHAIN=$BEST" -- --workload config3 --global-batch 8 $A || exit $?
cp gpurun_out/ab.log $OUT/ab_chain.txt
export TMPDIR=/tmp
rm -rf $OUT/prof
MSW_HOP_CHAIN=$BEST timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit $?
python3 tools/step_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/step_breakdown.txt
echo done >> $OUT/ab_chain.txt
