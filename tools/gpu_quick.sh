#!/bin/bash
# Short GPU-box check: GPU parity tests (verbose, per-test timeout) then a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -15
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 --cpu-budget 0 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -3 gpurun_out/bench.log
exit $(( rc > rc2 ? rc : rc2 ))
