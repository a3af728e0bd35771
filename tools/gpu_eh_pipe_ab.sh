#!/bin/bash
# Verdict r3 item 4 on the GPU box: the software-pipelined grid-stride edge MLP + hop (build
# variant ehpipe8: 8 waves per workgroup, 2 per SIMD, tile i+1's gathers + tile i+2's record
# in flight) -- bit identity against the default library, then a same-box A/B on config 5
# (hbm1m) interleaved twice, then a kernel trace of the variant on hbm1m.
#   bash tools/gpu_eh_pipe_ab.sh OUTDIR [VARIANT]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ehpipe}
V=${2:-ehpipe8}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread \
  -k "build_variant_matches_default" > $OUT/identity.log 2>&1 || exit 3
grep -q " passed" $OUT/identity.log || exit 3
: > gpurun_out/ab.log
export AB_KEEP=1
H="--workload hbm1m --no-cpu-baseline --no-roofline-large --steps 3 --warmup 1"
bash tools/ab.sh "" "MSW_LIB_VARIANT=$V" "" "MSW_LIB_VARIANT=$V" -- $H || exit 4
cp gpurun_out/ab.log $OUT/ab_hbm1m.txt
MSW_LIB_VARIANT=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv \
  -- python3 bench.py $H > $OUT/prof.json 2> $OUT/prof.err || exit 5
echo done >> $OUT/ab_hbm1m.txt
