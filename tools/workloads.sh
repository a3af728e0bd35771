#!/bin/bash
# Bench every BASELINE workload once on the GPU box (tools/gpu_session.sh style: own time
# limit per run, stop on a failure).  Output: gpurun_out/workloads.jsonl, one line per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/workloads.jsonl
run() {
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline-large "$@" > gpurun_out/wl_run.json 2> gpurun_out/wl_run.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$*] rc=$rc" >> gpurun_out/workloads.jsonl; tail -5 gpurun_out/wl_run.err >> gpurun_out/workloads.jsonl; exit $rc; fi
  python -c "import json,sys; d=json.load(open('gpurun_out/wl_run.json')); d['args']=sys.argv[1]; print(json.dumps({k:d[k] for k in ('args','value','ms_per_step','engine','parity') if k in d}))" "$*" >> gpurun_out/workloads.jsonl
}
run --steps 10 --warmup 3
run --workload zenodo4 --batch 8 --steps 10 --warmup 3
run --workload config3 --global-batch 8 --steps 10 --warmup 3
run --workload zenodo3 --steps 10 --warmup 3
run --workload zenodo4_k2f16 --steps 10 --warmup 3
run --workload zenodo4_f64 --steps 6 --warmup 2
run --workload dk15 --T 200 --steps 3 --warmup 1
run --workload hbm1m --T 100 --steps 2 --warmup 1
run --caller reference-loop --steps 3 --warmup 1
cat gpurun_out/workloads.jsonl
