#!/bin/bash
# A/B timing of engine variants on the GPU box: one bench run per environment setting.
#   bash tools/ab.sh "" "MSW_POOL_FUSE=0" "MSW_UNPOOL_FUSE=0" [-- bench args]
# Each run has its own time limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
envs=(); args=()
while [ $# -gt 0 ]; do
  if [ "$1" == "--" ]; then shift; args=("$@"); break; fi
  envs+=("$1"); shift
done
[ ${#args[@]} -eq 0 ] && args=(--no-cpu-baseline --steps 10 --warmup 3)
[ -z "${AB_KEEP:-}" ] && : > gpurun_out/ab.log
for e in "${envs[@]}"; do
  env $e timeout -k 10 300 python bench.py "${args[@]}" > gpurun_out/ab_run.json 2> gpurun_out/ab_run.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$e] rc=$rc" >> gpurun_out/ab.log; tail -5 gpurun_out/ab_run.err >> gpurun_out/ab.log; exit $rc; fi
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_run.json')); print('[%s]'%sys.argv[1], d['config']['workload'], 'B=%s'%d['config'].get('batch_per_gpu', d['config'].get('global_batch')), round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms', d['engine']['kernels_per_step'], 'launches', 'eh_us', round(list(d['roofline']['other_kernels'].values())[0]['avg_launch_us'],1), 'hop_us', round(d['roofline']['avg_launch_us'],1), 'parity', d.get('parity',{}).get('vs_reference_fixture',{}).get('max_rel_err'))" "$e" >> gpurun_out/ab.log
done
cat gpurun_out/ab.log
