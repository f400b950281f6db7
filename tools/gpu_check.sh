#!/bin/bash
# GPU-box check: GPU parity tests (verbose, per-test timeout, near-tie report) then a short bench.
# Every GPU step has its own time limit; a crash (rc > 1 from pytest) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/parity_report.jsonl
LG_PARITY_REPORT=gpurun_out/parity_report.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -25
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 --cpu-budget ${CPU_BUDGET:-0} ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -3 gpurun_out/bench.log
exit $(( rc > rc2 ? rc : rc2 ))
