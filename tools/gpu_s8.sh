set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_hip -o run --output-format csv -- python3 tools/train_bench.py --only hip --steps 3 --warmup 1 > $O/train_hip.json 2> $O/prof_hip.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_torch -o run --output-format csv -- python3 tools/train_bench.py --only torch --steps 3 --warmup 1 > $O/train_torch.json 2> $O/prof_torch.err || exit 6
echo ok
