# round-3 session R: same-box before / after of both fusions on the final tree (zenodo4)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03r; mkdir -p $O
bash tools/ab.sh "MSW_POOL_FUSE=0 MSW_UNPOOL_FUSE=0" "MSW_POOL_FUSE=1" "MSW_POOL_FUSE=0 MSW_UNPOOL_FUSE=0" "MSW_POOL_FUSE=1" "MSW_POOL_FUSE=0 MSW_UNPOOL_FUSE=0" "MSW_POOL_FUSE=1" > $O/ab.txt 2>&1 || exit 4
cp gpurun_out/ab.log $O/ab.log
cat $O/ab.log
