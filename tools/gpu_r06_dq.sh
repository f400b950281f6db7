#!/bin/bash
# Round 6: attention-backward dQ on fp16x3 (LG_TB_DQ_H3) -- training tests, then a same-box A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_dq; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_loss.py -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|worst" $O/pytest_train.log | cut -c1-300 | tail -25; [ $rc -ne 0 ] && exit $rc
ROUNDS=2 bash tools/ab_train.sh ab/dq0.so ab/dqh3.so 2>&1 | tee $O/ab_train.txt
