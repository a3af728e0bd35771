#!/bin/bash
# Round-4 A/B session: the persistent hop chains (MSW_HOP_CHAIN 0/1/2) first, then the
# software-pipelined grid-stride edge MLP + hop (build variant ehpipe8) on config 5.
# Each sub-script gives every GPU step its own time limit and stops at the first failure.
#   bash tools/gpu_ab_r04.sh [CHAIN_BEST]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab_r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -v -s --timeout 120 --timeout-method thread \
  -k "reference_fixture or autocast" > gpurun_out/ab_r04/train_tests.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "train tests rc=$rc"; exit 2; }
bash tools/gpu_chain_ab.sh chain ${1:-2} > gpurun_out/chain_ab.log 2>&1 || { echo "chain A/B rc=$?"; exit 3; }
bash tools/gpu_eh_pipe_ab.sh ehpipe ehpipe8 > gpurun_out/ehpipe_ab.log 2>&1 || { echo "ehpipe A/B rc=$?"; exit 4; }
echo done
