# round 5 session: SQ counters of the config-5 launches (hbm1m), three --pmc passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s16; mkdir -p $O
export TMPDIR=/tmp
B="python3 tools/pmc_step.py hbm1m 2"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
         "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $C -d $PWD/$O/pmc$i -o run --output-format csv -- $B > $O/pmc$i.log 2>&1 || exit $((10+i))
done
python3 tools/pmc_generic.py $O/pmc1 $O/pmc2 $O/pmc3 > $O/sq_hbm1m.txt 2>&1
