#!/bin/bash
# Round-4 closing session on the FINAL library: rocprofv3 kernel trace of bench.py (-> the
# roofline timing summary + step breakdown), the two PMC passes (-> HBM traffic summary), both
# copied into profiles/ on the box so that the closing bench line reads sources measured on
# the library it loads (roofline.rocprof / traffic_source: stale = false), then that bench
# line, the F = 64 and config-5 lines, a two-rank gloo rehearsal of the N > 1 line.  Every GPU
# step has its own time limit.
#   bash tools/gpu_final_r04.sh OUTDIR
set -u
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
rm -rf $OUT/prof $OUT/pmc_fetch $OUT/pmc_write
step rocprof 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
python3 tools/roofline_check.py $OUT/prof/run_kernel_trace.csv --json $OUT/roofline_rocprof.json > $OUT/roofline_check.txt 2>&1
python3 tools/step_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/step_breakdown.txt 2>&1
KRE='k_hop|k_edge_hop|k_pool|k_encode'
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc_write.log 2>&1
python3 tools/pmc_summary.py $OUT/pmc_summary.json $OUT/pmc_fetch $OUT/pmc_write > $OUT/pmc_summary.log 2>&1
cp $OUT/roofline_rocprof.json profiles/roofline_rocprof.json && cp $OUT/pmc_summary.json profiles/pmc_summary.json
step bench 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
step bench_f64 300 python bench.py --workload zenodo4_f64 --no-roofline-large > $OUT/bench_f64.json 2> $OUT/bench_f64.err
step bench_hbm1m 400 python bench.py --workload hbm1m --no-cpu-baseline --steps 3 --warmup 1 > $OUT/bench_hbm1m.json 2> $OUT/bench_hbm1m.err
# the N > 1 path rehearsed on the one-GPU box: two ranks over gloo sharing cuda:0, the
# post-timed extras inside one --extras-budget (per-section wall_s, skipped sections marked)
step rehearsal 420 env MSW_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --extras-budget 180 > $OUT/rehearsal_2rank_gloo.json 2> $OUT/rehearsal_2rank_gloo.err
echo done >> $OUT/steps.log
