#!/bin/bash
# Round 6: input preparation without the descriptor copy + one-launch range pass -- GPU suite, then a
# same-box A/B against the previous build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_prep; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -8; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 bash tools/ab_bench.sh ab/head.so ab/cur.so 2>&1 | tee $O/ab_bench.txt
