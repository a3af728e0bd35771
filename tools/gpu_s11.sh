set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s11; mkdir -p $O
for v in 1 2; do
  for wl in "--workload config3 --global-batch 8" "--workload zenodo4" "--workload dk15 --T 200"; do
    MSW_HOP_ROWS=$v timeout -k 10 300 python bench.py $wl --no-cpu-baseline --no-roofline-large --steps 10 --warmup 3 > $O/tmp.json 2>> $O/err.log || exit 5
    python -c "
import json,sys; d=json.loads(open('$O/tmp.json').read().strip().splitlines()[-1]); print(json.dumps({'rows':'$v','wl':'$wl','value':d['value'],'ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
echo ok
