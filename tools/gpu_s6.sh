set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s6; mkdir -p $O
for v in "" rfl rfl4 rdc2; do
  MSW_LIB_VARIANT=$v timeout -k 10 300 python tools/ab_hop_rows.py --settings 0 1 >> $O/ab_rows.jsonl 2>> $O/ab.err || exit 5
done
echo ok
