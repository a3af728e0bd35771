set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "row_layout" > $O/rows_tests.log 2>&1 || exit 4
timeout -k 10 300 python tools/ab_hop_rows.py --settings 0 1 > $O/ab_rows_dc4.jsonl 2> $O/ab.err || exit 5
MSW_LIB_VARIANT=rdc3 timeout -k 10 300 python tools/ab_hop_rows.py --settings 0 1 > $O/ab_rows_dc3.jsonl 2>> $O/ab.err || exit 6
MSW_LIB_VARIANT=rdc2 timeout -k 10 300 python tools/ab_hop_rows.py --settings 0 1 > $O/ab_rows_dc2.jsonl 2>> $O/ab.err || exit 7
echo ok
