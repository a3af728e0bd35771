#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel trace of the bench.
# Every GPU step has its own time limit; a fault / abort / timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/steps.log
step() {  # step NAME SECONDS CMD...  (exit codes 0/1 continue; anything else stops)
  local name=$1 secs=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >> $OUT/steps.log; exit $rc; fi
}
MODE=${1:-all}
if [[ $MODE == all || $MODE == tests ]]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  if ! grep -q "smoke ok" $OUT/smoke.log; then echo "stopping: smoke failed" >> $OUT/steps.log; exit 3; fi
  step gputests 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
fi
if [[ $MODE == all || $MODE == prof ]]; then
  export TMPDIR=/tmp
  rm -rf $OUT/prof
  step rocprof 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
fi
if [[ $MODE == all || $MODE == extra ]]; then
  step bench_refloop 300 python bench.py --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1 > $OUT/bench_refloop.json 2> $OUT/bench_refloop.err
  step bench_config3 300 python bench.py --workload config3 --global-batch 8 --no-roofline-large --steps 5 --warmup 2 > $OUT/bench_config3.json 2> $OUT/bench_config3.err
  [[ -n "${STRONG:-}" ]] && step strong 900 python tools/strong_scaling.py --workload config3 --G 8 20 64 > $OUT/strong_scaling.jsonl 2> $OUT/strong_scaling.err
fi
if [[ $MODE == pmc ]]; then
  export TMPDIR=/tmp
  rm -rf $OUT/pmc_fetch $OUT/pmc_write
  KRE='k_hop|k_edge_hop|k_pool|k_encode'
  step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1
  step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc_write.log 2>&1
  python3 tools/pmc_summary.py $OUT/pmc_summary.json $OUT/pmc_fetch $OUT/pmc_write > $OUT/pmc_summary.log 2>&1
fi
if [[ $MODE == trace ]]; then
  step trace 300 python tools/trace_kernels.py > $OUT/trace.log 2>&1
fi
echo done >> $OUT/steps.log
