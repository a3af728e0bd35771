# round 5 session: DMA edge hop at four waves per workgroup (bit identity + A/B on hbm1m),
# encoder-prefetch build variant bit identity at zenodo4 F = 64
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s13; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread -k "dma_edge or build_variant" > $O/tests.log 2>&1 || exit 3
bash tools/ab.sh "" "MSW_EH_DMA=1" "MSW_EH_DMA=2" "" "MSW_EH_DMA=1" "MSW_EH_DMA=2" -- --workload hbm1m --no-cpu-baseline --steps 5 --warmup 2 || exit 4
cp gpurun_out/ab.log $O/ab_hbm1m.log
