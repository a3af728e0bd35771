#!/bin/bash
# Round-6 GPU sessions, one script with modes (replaces the round-5 one-off tools/gpu_r05_s*.sh).
#   bash tools/gpu_r06.sh MODE [OUTDIR] [args...]
# Modes:
#   rccl        the one-rank RCCL tests (tests/test_gpu_rccl.py) + the partitioned-rollout tests
#   train       the HIP training-gradient tests (tests/test_gpu_train.py)
#   tests       the whole -m gpu suite and smoke()
#   pytest      pytest -m gpu on the test ids given as args
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
    # (the nofastdiv variant predates the hop chains: MSW_HOP_WG=0 on the default library)
    step ab_hbm1m 900 bash tools/ab.sh "MSW_HOP_WG=0" "MSW_LIB_VARIANT=nofastdiv" "MSW_HOP_WG=0" "MSW_LIB_VARIANT=nofastdiv" -- --workload hbm1m --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1
    cp gpurun_out/ab.log $OUT/ab_hbm1m.txt
    step ab_zenodo4 600 bash tools/ab.sh "MSW_HOP_WG=0" "MSW_LIB_VARIANT=nofastdiv" "MSW_HOP_WG=0" "MSW_LIB_VARIANT=nofastdiv" "MSW_HOP_WG=0" "MSW_LIB_VARIANT=nofastdiv"
    cp gpurun_out/ab.log $OUT/ab_zenodo4.txt ;;
  chain)  # one-workgroup hop chains: bit identity, then the A/B on zenodo4 and the batch of 8
    step chain_tests 600 $PYT tests/test_gpu_parity.py -m gpu -k "hop_chain or partitioned or group_rollout" > $OUT/chain_tests.txt 2>&1
    step ab_chain 900 bash tools/ab.sh "MSW_HOP_WG=0" "MSW_HOP_WG=1" "MSW_HOP_WG=2" "MSW_HOP_WG=0" "MSW_HOP_WG=1" "MSW_HOP_WG=2"
    cp gpurun_out/ab.log $OUT/ab_chain_zenodo4.txt ;;
  cputhreads)
    step cpu_threads 600 python tools/cpu_threads.py > $OUT/cpu_threads.json 2> $OUT/cpu_threads.err ;;
  *)
    echo "unknown mode $MODE" >&2; exit 2 ;;
esac
echo done >> $OUT/steps.log
