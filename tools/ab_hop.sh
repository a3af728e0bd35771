#!/bin/bash
# A/B of library variants on config 5 (hbm1m): whole-rollout rate and the finest middle hop's
# roofline numbers (bench.py roofline: HIP-event timed launches).  Usage: bash tools/ab_hop.sh v1 v2 ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/ab_hop.log
for v in "$@"; do
  [ "$v" == "-" ] && v=""
  MSW_LIB_VARIANT=$v timeout -k 10 300 python bench.py --workload hbm1m --T 20 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_hop.json 2> gpurun_out/ab_hop.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$v] rc=$rc" >> gpurun_out/ab_hop.log; tail -5 gpurun_out/ab_hop.err >> gpurun_out/ab_hop.log; exit $rc; fi
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_hop.json')); r=d['roofline']; print('[%s]'%sys.argv[1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; hop', round(r['avg_launch_us'],1), 'us', round(r['achieved']), 'GB/s frac', round(r['frac'],3))" "$v" >> gpurun_out/ab_hop.log
done
cat gpurun_out/ab_hop.log
