#!/bin/bash
# Round-4 GPU-box sessions behind profiles/r04/ (one file, one function per session; the
# closing profile session is tools/gpu_final_r04.sh).  Every GPU step has its own time limit.
#   bash tools/gpu_r04_sessions.sh MODE [OUTDIR]
#   MODE: f64-sweep  -- F = 64 step breakdown + plan-switch A/B (profiles/r04/ab_f64_switches.txt)
#         ldsw       -- LDS-typed vs FLAT MLP operands at F = 64 (profiles/r04/ab_f64_lds_operands.txt)
#         sq-f64     -- SQ counters of the F = 64 step (profiles/r04/pmc_sq_f64_flat.txt)
#         close-tests -- smoke, the -m gpu suite, F = 64 step breakdown on the final library
#         close-lines -- bench lines of configs 3 / 4, the reference loop, the training bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
MODE=${1:?mode}
shift

f64_sweep() {
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
}

ldsw() {
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
}

sq_f64() {
  O=gpurun_out/sqf64; mkdir -p $O; export TMPDIR=/tmp
  KRE='k_edge_mlp|k_encode|k_edge_coop4|k_hop_split'
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVES --kernel-include-regex "$KRE" -d $PWD/$O/pmc_sq -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 1 --warmup 1 > $O/pmc_sq.log 2>&1 || exit 3
  timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$KRE" -d $PWD/$O/pmc_grbm -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 1 --warmup 1 > $O/pmc_grbm.log 2>&1 || exit 4
  python3 tools/pmc_generic.py $O/pmc_sq $O/pmc_grbm > $O/pmc_generic.txt 2>&1
}

close_tests() {
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
}

close_lines() {
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
}

case "$MODE" in
  f64-sweep) f64_sweep "$@" ;;
  ldsw) ldsw "$@" ;;
  sq-f64) sq_f64 "$@" ;;
  close-tests) close_tests "$@" ;;
  close-lines) close_lines "$@" ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
