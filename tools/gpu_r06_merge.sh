#!/bin/bash
# Round 6: two-image launches for the positional encoding, the descriptor planes and the final
# matchability -- GPU suite, then same-box A/Bs at configs[2] and at configs[1] (B = 1, N = 1024)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_merge; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -8; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 bash tools/ab_bench.sh ab/head.so ab/cur.so 2>&1 | tee $O/ab_cfg2.txt
ROUNDS=3 STEPS=200 BENCH_ARGS="--batch 1 --npts 1024" bash tools/ab_bench.sh ab/head.so ab/cur.so 2>&1 | tee $O/ab_cfg1.txt
