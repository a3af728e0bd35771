#!/bin/bash
# Closing check on the final library: smoke, the whole -m gpu suite, the F = 64 step breakdown.
#   bash tools/gpu_close_tests.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-close}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $OUT/bench_prof_f64.json 2> $OUT/bench_prof_f64.err || exit 4
python3 tools/step_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/step_breakdown_f64.txt
rm -rf $OUT/prof
echo done > $OUT/done
