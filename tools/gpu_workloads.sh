#!/bin/bash
# GPU box: bench.py on every workload (one rank) -> gpurun_out/workloads.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/workloads.jsonl
for w in ${WORKLOADS:-configs2 configs3 configs4}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-10} --warmup 2 --cpu-budget 0 > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "$w rc=$rc"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_$w.log; exit $rc; }
  grep '^{' gpurun_out/bench_$w.log >> gpurun_out/workloads.jsonl
done
