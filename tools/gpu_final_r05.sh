#!/bin/bash
# Round-5 closing session on the library in the tree: the -m gpu suite and smoke(), the
# rocprofv3 kernel trace of bench.py (-> roofline timing summary + zenodo4 step breakdown), the
# two PMC passes (-> HBM traffic summary), copied into profiles/ on the box so that the bench
# line that follows reads sources measured on the library it loads (stale = false); the F = 64
# trace + step breakdown; the bench lines of every workload; the training bench; the N > 1
# path rehearsed on the one-GPU box (bench.py --gpus 2 starting its own two gloo ranks).
# Every GPU step has its own time limit; a step that fails other than with rc 1 stops it.
# Two calls (each within gpurun's 20-minute limit); copy part a's roofline_rocprof.json and
# pmc_summary.json into profiles/ before part b, so that its lines read them too.
#   bash tools/gpu_final_r05.sh OUTDIR a|b
set -u
PART=${2:-a}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
: > $OUT/steps.log
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...  (exit codes 0/1 continue; anything else stops)
  local name=$1 secs=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >> $OUT/steps.log; exit $rc; fi
}
if [ $PART == a ]; then
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rm -rf $OUT/prof $OUT/prof_f64 $OUT/pmc_fetch $OUT/pmc_write
step rocprof 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
python3 tools/roofline_check.py $OUT/prof/run_kernel_trace.csv --json $OUT/roofline_rocprof.json > $OUT/roofline_check.txt 2>&1
python3 tools/step_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/step_breakdown.txt 2>&1
KRE='k_hop|k_edge_hop|k_pool|k_encode'
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc_write.log 2>&1
python3 tools/pmc_summary.py $OUT/pmc_summary.json $OUT/pmc_fetch $OUT/pmc_write > $OUT/pmc_summary.log 2>&1
cp $OUT/roofline_rocprof.json profiles/roofline_rocprof.json && cp $OUT/pmc_summary.json profiles/pmc_summary.json
step bench 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
else
step rocprof_f64 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_f64 -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $OUT/bench_f64_prof.json 2> $OUT/bench_f64_prof.err
python3 tools/step_breakdown.py $OUT/prof_f64/run_kernel_trace.csv > $OUT/step_breakdown_f64.txt 2>&1
step bench_f64 300 python bench.py --workload zenodo4_f64 --no-roofline-large > $OUT/bench_f64.json 2> $OUT/bench_f64.err
step bench_hbm1m 400 python bench.py --workload hbm1m --no-cpu-baseline --steps 3 --warmup 1 > $OUT/bench_hbm1m.json 2> $OUT/bench_hbm1m.err
step refloop 300 python bench.py --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1 > $OUT/bench_refloop.json 2> $OUT/bench_refloop.err
step config3 300 python bench.py --workload config3 --global-batch 8 --no-roofline-large --steps 5 --warmup 2 > $OUT/bench_config3.json 2> $OUT/bench_config3.err
step dk15 300 python bench.py --workload dk15 --T 200 --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1 > $OUT/bench_dk15.json 2> $OUT/bench_dk15.err
step train_bench 300 python tools/train_bench.py --amp --fp64-ref > $OUT/train_bench.json 2> $OUT/train_bench.err
step rehearsal 420 env MSW_DIST_BACKEND=gloo python bench.py --gpus 2 --extras-budget 180 > $OUT/rehearsal_2rank_gloo.json 2> $OUT/rehearsal_2rank_gloo.err
fi
echo done >> $OUT/steps.log
