# round 5 session: cooperative encoder with operands issued ahead -- bit identity, A/B, trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s12; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "coop_encoder or deferred_decoder" > $O/tests.log 2>&1 || exit 3
AB_KEEP= bash tools/ab.sh "" "MSW_LIB_VARIANT=encpf0" "" "MSW_LIB_VARIANT=encpf0" -- --workload zenodo4_f64 --no-cpu-baseline --steps 20 --warmup 3 || exit 4
cp gpurun_out/ab.log $O/ab_f64.log
timeout -k 10 240 env MSW_TRACE_ENCODE=1 MSW_LIB_VARIANT=trace python -u tools/trace_kernels.py zenodo4_f64 > $O/trace_f64.txt 2>&1 || exit 5
