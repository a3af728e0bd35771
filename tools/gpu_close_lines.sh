#!/bin/bash
# Closing bench lines of the other BASELINE configs on the final library + the training
# benchmark.   bash tools/gpu_close_lines.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-lines}
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
step config3 300 python bench.py --workload config3 --global-batch 8 --no-roofline-large --steps 5 --warmup 2 > $OUT/bench_config3.json 2> $OUT/bench_config3.err
step dk15 300 python bench.py --workload dk15 --T 200 --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1 > $OUT/bench_dk15.json 2> $OUT/bench_dk15.err
step refloop 300 python bench.py --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1 > $OUT/bench_refloop.json 2> $OUT/bench_refloop.err
step train_bench 300 python tools/train_bench.py --amp --fp64-ref > $OUT/train_bench.json 2> $OUT/train_bench.err
echo done >> $OUT/steps.log
