#!/bin/bash
# F = 64 MLP operands through an LDS-typed pointer (default) vs the round-3 generic pointer
# (build variant flatw): F = 64 parity tests + bit identity of the variants, then a same-box
# A/B on zenodo4_f64 and zenodo4, then a kernel trace of the F = 64 step.
#   bash tools/gpu_ldsw_ab.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ldsw}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread \
  -k "64 or build_variant" > $OUT/tests.log 2>&1
rc=$?; [ $rc -ne 0 ] && { echo "tests rc=$rc" >> $OUT/steps.log; exit 3; }
export AB_KEEP=1
: > gpurun_out/ab.log
A="--no-cpu-baseline --no-roofline-large --steps 10 --warmup 3"
bash tools/ab.sh "" "MSW_MLP_PIPE=0" "MSW_LIB_VARIANT=flatw" "" "MSW_MLP_PIPE=0" "MSW_LIB_VARIANT=flatw" -- --workload zenodo4_f64 $A || exit 4
bash tools/ab.sh "" "MSW_LIB_VARIANT=flatw" -- $A || exit 5
cp gpurun_out/ab.log $OUT/ab_ldsw.txt
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 6
python3 tools/step_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/step_breakdown_f64.txt
echo done >> $OUT/ab_ldsw.txt
