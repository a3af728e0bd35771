#!/bin/bash
# Round-6 GPU sessions, one script with modes (replaces the round-5 one-off tools/gpu_r05_s*.sh).
#   bash tools/gpu_r06.sh MODE [OUTDIR] [args...]
# Modes:
#   rccl        the one-rank RCCL tests (tests/test_gpu_rccl.py) + the partitioned-rollout tests
#   train       the HIP training-gradient tests (tests/test_gpu_train.py)
#   tests       the whole -m gpu suite and smoke()
#   schedfuzz   tests/test_gpu_schedule_fuzz.py over a seed range (SCHED_FUZZ_SEEDS, default 0:200)
#   partfuzz    tests/test_gpu_partition_fuzz.py over a seed range (PART_FUZZ_SEEDS, default 0:200)
#   trainfuzz   tests/test_gpu_train_fuzz.py over a seed range (TRAIN_FUZZ_SEEDS, default 0:300)
#   pmc5        HBM bytes per launch of config 5's kernels (FETCH_SIZE / WRITE_SIZE passes)
#   stream      streaming stores of the large-mesh encoder / row hop: bit-identity, parity, A/B, trace
#   pytest      pytest -m gpu on the test ids given as args
#   fuzz        tests/test_gpu_fuzz.py over a wider seed range (FUZZ_SEEDS, default 16:400)
#   ab          tools/ab.sh with the args (A/B of MSW_* settings on bench.py)
#   bench       bench.py with the args
#   prof        rocprofv3 kernel trace of bench.py with the args (+ step breakdown)
#   sq          SQ counter pass(es) of bench.py with the args, one rocprofv3 run per counter set
# Every GPU step has its own time limit; a step that fails other than with rc 1 stops the call.
set -u
MODE=${1:?mode}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${2:-$MODE}
shift $(( $# >= 2 ? 2 : $# ))
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
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
case $MODE in
  rccl)
    step rccl 400 $PYT tests/test_gpu_rccl.py tests/test_gpu_parity.py -k "rccl or nccl or self_exchange or partitioned or group_rollout" -m gpu > $OUT/rccl_tests.txt 2>&1 ;;
  train)
    step train 900 $PYT tests/test_gpu_train.py -m gpu > $OUT/train_tests.txt 2>&1 ;;
  tests)
    step tests 1000 $PYT tests -m gpu > $OUT/gpu_tests.txt 2>&1
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
  fuzz)  # a wider seed range of tests/test_gpu_fuzz.py (args: the range, default 16:400)
    export FUZZ_SEEDS=${1:-16:400}; step fuzz 1000 $PYT -m gpu tests/test_gpu_fuzz.py > $OUT/fuzz.txt 2>&1 ;;
  schedfuzz)  # tests/test_gpu_schedule_fuzz.py over a seed range (args: the range, default 0:200)
    export SCHED_FUZZ_SEEDS=${1:-0:200}; step schedfuzz 1000 $PYT -m gpu tests/test_gpu_schedule_fuzz.py > $OUT/schedfuzz.txt 2>&1 ;;
  partfuzz)  # tests/test_gpu_partition_fuzz.py over a seed range (args: the range, default 0:200)
    export PART_FUZZ_SEEDS=${1:-0:200}; step partfuzz 1000 $PYT -m gpu tests/test_gpu_partition_fuzz.py > $OUT/partfuzz.txt 2>&1 ;;
  trainfuzz)  # tests/test_gpu_train_fuzz.py over a seed range (args: the range, default 0:300)
    export TRAIN_FUZZ_SEEDS=${1:-0:300}; step trainfuzz 1000 $PYT -m gpu tests/test_gpu_train_fuzz.py > $OUT/trainfuzz.txt 2>&1 ;;
  pmc5)  # HBM bytes per launch of config 5's kernels (FETCH_SIZE / WRITE_SIZE, separate passes)
    KRE='k_encode|k_edge_hop|k_hop|k_pool|k_epi'
    step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --workload hbm1m --no-cpu-baseline --no-roofline-large --steps 1 --warmup 1 > $OUT/pmc_fetch.log 2>&1
    step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_write -o run --output-format csv -- python3 bench.py --workload hbm1m --no-cpu-baseline --no-roofline-large --steps 1 --warmup 1 > $OUT/pmc_write.log 2>&1
    python3 tools/pmc_summary.py $OUT/pmc_summary_hbm1m.json $OUT/pmc_fetch $OUT/pmc_write > $OUT/pmc_summary.log 2>&1 ;;
  stream)  # streaming stores of the large-mesh encoder / row hop + the encoder's input prefetch:
           # variant bit-identity (nostream = the closing-session kernels), parity, A/B, trace
    step variants 600 $PYT tests/test_gpu_parity.py -m gpu -k "build_variant or row_layout or coop_encoder" > $OUT/variants.txt 2>&1
    step fullsize 600 $PYT -m gpu tests/test_gpu_fullsize.py -k config5 > $OUT/fullsize.txt 2>&1
    step ab_hbm1m 900 bash tools/ab.sh "" "MSW_LIB_VARIANT=nostream" "" "MSW_LIB_VARIANT=nostream" -- --workload hbm1m --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1
    cp gpurun_out/ab.log $OUT/ab_hbm1m.txt
    step ab_zenodo4 600 bash tools/ab.sh "" "MSW_LIB_VARIANT=nostream" "" "MSW_LIB_VARIANT=nostream"
    cp gpurun_out/ab.log $OUT/ab_zenodo4.txt
    rm -rf $OUT/prof
    step rocprof 500 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --workload hbm1m --no-roofline-large --steps 3 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
    python3 tools/step_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/step_breakdown_hbm1m.txt 2>&1 ;;
  pytest)
    step pytest 900 $PYT -m gpu "$@" > $OUT/pytest.txt 2>&1 ;;
  ab)
    step ab 1000 bash tools/ab.sh "$@"
    cp gpurun_out/ab.log $OUT/ab.log ;;
  bench)
    step bench 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err ;;
  prof)
    rm -rf $OUT/prof
    step rocprof 500 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $OUT/bench_prof.json 2> $OUT/bench_prof.err
    python3 tools/step_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/step_breakdown.txt 2>&1 ;;
  divab)  # the shared-reciprocal division: exactness sweep, bit-identity of the variants, A/B
    step div_check 120 ./tools/div_check > $OUT/div_check.txt 2>&1
    step variants 600 $PYT tests/test_gpu_parity.py -m gpu -k "build_variant" > $OUT/variants.txt 2>&1
    step ab_hbm1m 900 bash tools/ab.sh "" "MSW_LIB_VARIANT=nofastdiv" "" "MSW_LIB_VARIANT=nofastdiv" -- --workload hbm1m --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1
    cp gpurun_out/ab.log $OUT/ab_hbm1m.txt
    step ab_zenodo4 600 bash tools/ab.sh "" "MSW_LIB_VARIANT=nofastdiv" "" "MSW_LIB_VARIANT=nofastdiv" "" "MSW_LIB_VARIANT=nofastdiv"
    cp gpurun_out/ab.log $OUT/ab_zenodo4.txt ;;
  sq)  # SQ counters of config 5's fused edge MLP + hop, per launch (tools/pmc_generic.py --split-duration)
    KRE=${SQ_KRE:-k_edge_hop}
    C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
    C2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
    C3="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES"
    i=0
    for C in "$C1" "$C2" "$C3"; do
      i=$((i+1)); rm -rf $OUT/sq$i
      step sq$i 240 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d $PWD/$OUT/sq$i -o run --output-format csv -- python3 tools/pmc_step.py hbm1m 2 > $OUT/sq$i.log 2>&1
    done
    python3 tools/pmc_generic.py --split-duration $OUT/sq1 $OUT/sq2 $OUT/sq3 > $OUT/sq_hbm1m.txt 2>&1 ;;
  final-a)  # closing session, part a: the -m gpu suite and smoke(), the rocprofv3 kernel trace of
            # bench.py (-> roofline timing summary + step breakdown), the two PMC passes (-> HBM
            # traffic summary), copied into profiles/ so that the bench line after them reads
            # summaries measured on the library it loads
    step tests 1000 $PYT tests -m gpu > $OUT/gpu_tests.txt 2>&1
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
    rm -rf $OUT/prof $OUT/pmc_fetch $OUT/pmc_write
    step rocprof 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
    python3 tools/roofline_check.py $OUT/prof/run_kernel_trace.csv --json $OUT/roofline_rocprof.json > $OUT/roofline_check.txt 2>&1
    python3 tools/step_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/step_breakdown.txt 2>&1
    KRE='k_hop|k_edge_hop|k_pool|k_encode'
    step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1
    step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $PWD/$OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc_write.log 2>&1
    python3 tools/pmc_summary.py $OUT/pmc_summary.json $OUT/pmc_fetch $OUT/pmc_write > $OUT/pmc_summary.log 2>&1
    cp $OUT/roofline_rocprof.json profiles/roofline_rocprof.json && cp $OUT/pmc_summary.json profiles/pmc_summary.json
    step bench 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err ;;
  final-b)  # part b: the other workloads' lines, F = 64 trace, the CPU thread sweep, the N > 1 rehearsal
    rm -rf $OUT/prof_f64
    step rocprof_f64 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_f64 -o run --output-format csv -- python3 bench.py --workload zenodo4_f64 --no-cpu-baseline --no-roofline-large --steps 5 --warmup 1 > $OUT/bench_f64_prof.json 2> $OUT/bench_f64_prof.err
    python3 tools/step_breakdown.py $OUT/prof_f64/run_kernel_trace.csv > $OUT/step_breakdown_f64.txt 2>&1
    step bench_f64 300 python bench.py --workload zenodo4_f64 --no-roofline-large > $OUT/bench_f64.json 2> $OUT/bench_f64.err
    step bench_hbm1m 400 python bench.py --workload hbm1m --no-cpu-baseline --steps 3 --warmup 1 > $OUT/bench_hbm1m.json 2> $OUT/bench_hbm1m.err
    step refloop 300 python bench.py --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1 > $OUT/bench_refloop.json 2> $OUT/bench_refloop.err
    step config3 400 python bench.py --workload config3 --global-batch 8 --no-roofline-large --steps 5 --warmup 2 > $OUT/bench_config3.json 2> $OUT/bench_config3.err
    step dk15 300 python bench.py --workload dk15 --T 200 --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1 > $OUT/bench_dk15.json 2> $OUT/bench_dk15.err
    step cpu_threads 400 python tools/cpu_threads.py > $OUT/cpu_threads.json 2> $OUT/cpu_threads.err
    step rehearsal 420 env MSW_DIST_BACKEND=gloo python bench.py --gpus 2 --extras-budget 180 > $OUT/rehearsal_2rank_gloo.json 2> $OUT/rehearsal_2rank_gloo.err ;;
  final-c)  # part c: the config-3 line (CPU batch leg), the CPU thread sweep, the N > 1 rehearsal
    step config3 400 python bench.py --workload config3 --global-batch 8 --no-roofline-large --steps 5 --warmup 2 > $OUT/bench_config3.json 2> $OUT/bench_config3.err
    step cpu_threads 300 python -u tools/cpu_threads.py > $OUT/cpu_threads.json 2> $OUT/cpu_threads.err
    step rehearsal 420 env MSW_DIST_BACKEND=gloo python bench.py --gpus 2 --extras-budget 180 > $OUT/rehearsal_2rank_gloo.json 2> $OUT/rehearsal_2rank_gloo.err ;;
  cputhreads)
    step cpu_threads 600 python tools/cpu_threads.py > $OUT/cpu_threads.json 2> $OUT/cpu_threads.err ;;
  *)
    echo "unknown mode $MODE" >&2; exit 2 ;;
esac
echo done >> $OUT/steps.log
