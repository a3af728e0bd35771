set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s1; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "captured_forward or fused_rollout_matches or batch_vs_reference or single_step" > $O/gpu_tests_new.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --caller reference-loop --no-cpu-baseline --no-roofline-large --steps 5 --warmup 2 > $O/bench_refloop.json 2> $O/bench_refloop.err || exit 5
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || exit 6
MSW_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --strong-sets 8,128 > $O/rehearsal2.json 2> $O/rehearsal2.err || exit 7
echo ok
