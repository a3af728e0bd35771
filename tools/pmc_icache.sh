#!/bin/bash
# Instruction-cache / instruction-mix counters of the bench's kernels (one PMC pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1
grep -i -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_SMEM\|SQ_WAIT_INST_ANY\|SQ_WAVE_CYCLES\|SQ_BUSY_CYCLES" gpurun_out/pmc_list.txt | sort -u > gpurun_out/pmc_icache_avail.txt
cat gpurun_out/pmc_icache_avail.txt
rm -rf gpurun_out/pmc_ic
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES SQ_INSTS_SALU} --kernel-include-regex 'k_hop|k_edge_hop|k_pool|k_encode' -d $PWD/gpurun_out/pmc_ic -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmc_ic.log 2>&1
echo "rc=$?"
