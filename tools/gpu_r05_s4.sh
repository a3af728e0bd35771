set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "deferred_decoder or dma_edge_hops or captured_forward or speculative" > gpurun_out/s4/tests.log 2>&1 || exit 3
AB_KEEP= bash tools/ab.sh "MSW_DEFER_DECODE=0" "" "MSW_DEFER_DECODE=0" "" -- --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 5 --warmup 2 || exit 4
cp gpurun_out/ab.log gpurun_out/s4/ab_refloop.log
timeout -k 10 300 python -u tools/grad_layer_diag.py --R 1 --hip-calls 4 > gpurun_out/s4/layer_mixed4.jsonl 2> gpurun_out/s4/layer.err || exit 5
