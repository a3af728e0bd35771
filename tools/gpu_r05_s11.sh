# round 5 session: group-graph / DMA / decoder parity tests, partition bench graph vs eager
set -o pipefail
O=gpurun_out/s11; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "partition or group_rollout or dma_edge or deferred_decoder" > $O/tests.log 2>&1 || exit 3
for wl in zenodo4 hbm1m; do
  T=24; [ $wl == hbm1m ] && T=10
  timeout -k 10 300 python -u tools/partition_bench.py --workload $wl --T $T --parts 2 4 > $O/part_${wl}_graph.json 2> $O/part_${wl}_graph.err || exit 4
  timeout -k 10 300 python -u tools/partition_bench.py --workload $wl --T $T --parts 2 4 --eager > $O/part_${wl}_eager.json 2> $O/part_${wl}_eager.err || exit 5
done
