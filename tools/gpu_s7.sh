set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s7; mkdir -p $O
for v in "" rpipe rpipe4; do
  MSW_LIB_VARIANT=$v timeout -k 10 300 python tools/ab_hop_rows.py --settings 1 >> $O/ab_rows.jsonl 2>> $O/ab.err || exit 5
done
timeout -k 10 300 python bench.py --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 10 --warmup 2 > $O/bench_refloop.json 2> $O/bench_refloop.err || exit 6
timeout -k 10 600 python tools/train_bench.py > $O/train_bench.json 2> $O/train_bench.err || exit 7
echo ok
