# round-3 session H: A/B of wave-lockstep breakers in the grid-stride fused edge MLP + hop
# (config 5, hbm1m): static priority / delayed start of the younger half of each CU's waves
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03h; mkdir -p $O
export TMPDIR=/tmp
: > $O/ab.txt
for v in "" ehp1 ehs2 ehs6 ""; do
  MSW_LIB_VARIANT=$v timeout -k 10 300 python bench.py --workload hbm1m --no-cpu-baseline --steps 3 --warmup 1 > $O/b_$v.json 2> $O/b_$v.err || exit 5
  python -c "import json,sys; d=json.load(open(sys.argv[2])); lm=d['roofline'].get('large_mesh') or {}; print('[%s]'%sys.argv[1], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms', json.dumps(lm)[:600])" "$v" $O/b_$v.json >> $O/ab.txt
done
cat $O/ab.txt
