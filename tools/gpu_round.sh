#!/bin/bash
# One GPU session of this round: smoke, the -m gpu suite, bench (default workload), the
# training benchmark with its AMP leg.  Each GPU step has its own time limit; a fault / abort /
# time-out ends the session (tools/gpu_session.sh adds rocprof / PMC modes).
#   bash tools/gpu_round.sh OUTDIR [FIRST_TEST_EXPR]
# FIRST_TEST_EXPR: a pytest -k expression run on its own before everything else (new kernels)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04}
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
if [ -n "${2:-}" ]; then
  step first 240 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -k "$2" > $OUT/first.log 2>&1
  if ! grep -q " passed" $OUT/first.log || grep -q "failed" $OUT/first.log; then echo "stopping: first tests failed" >> $OUT/steps.log; exit 4; fi
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
step gputests 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
step bench 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
step train_bench 300 python tools/train_bench.py --amp --fp64-ref > $OUT/train_bench.json 2> $OUT/train_bench.err
echo done >> $OUT/steps.log
